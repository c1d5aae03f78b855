// spcg_plan.cpp — host plan of the point-sharded matrix-free PCG (spcg.h) for one rank.
//
// Input: the flattened graph arapOptimization builds (g2oBundleAdjustment.cc:640-953: per KF pair
// its reprojection / depth edges and the directed ARAP edges (p1_i, p2_i, p1_j, p2_j, T_g)).  All
// passes are O(E + P) counting sorts and scans, so a 500k x 8-keyframe graph (84M ARAP edges,
// SURVEY §8d C4) plans in seconds; nothing here depends on a fill-reducing ordering.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <functional>
#include <numeric>
#include <thread>

#include "host_threads.h"
#include "spcg.h"

namespace deftri {

namespace {

// stable counting sort of `ids` by key(id) in [0, nkeys)
template <class Key>
void counting_sort(std::vector<int32_t> &ids, int64_t nkeys, Key key) {
    std::vector<int64_t> cnt((size_t)nkeys + 1, 0);
    for (int32_t i : ids) cnt[(size_t)key(i) + 1]++;
    for (int64_t k = 0; k < nkeys; k++) cnt[k + 1] += cnt[k];
    std::vector<int32_t> out(ids.size());
    for (int32_t i : ids) out[(size_t)cnt[(size_t)key(i)]++] = i;
    ids.swap(out);
}

// the offsets of a chunked counting sort, key-major with chunk order inside a key: cnt[c][k] becomes
// chunk c's first write position for key k, key_start[k] (optional, nkeys + 1) key k's start. Key
// ranges on host threads: their totals, a prefix over the ranges, then each range's offsets
template <class T>
int64_t chunk_offsets(std::vector<std::vector<T>> &cnt, int64_t nkeys, int64_t *key_start) {
    const int64_t nch = (int64_t)cnt.size();
    const int64_t nkr = std::max<int64_t>(1, std::min<int64_t>(16, nkeys / (1 << 16)));
    auto k_of = [&](int64_t r) { return nkeys * r / nkr; };
    std::vector<int64_t> rbase((size_t)nkr + 1, 0);
    chunked(nkr, 1, [&](int, int64_t r0, int64_t r1) {
        for (int64_t r = r0; r < r1; r++) {
            int64_t t = 0;
            for (int64_t c = 0; c < nch; c++)
                for (int64_t k = k_of(r); k < k_of(r + 1); k++) t += cnt[c][k];
            rbase[r + 1] = t;
        }
    });
    for (int64_t r = 0; r < nkr; r++) rbase[r + 1] += rbase[r];
    chunked(nkr, 1, [&](int, int64_t r0, int64_t r1) {
        for (int64_t r = r0; r < r1; r++) {
            int64_t run = rbase[r];
            for (int64_t k = k_of(r); k < k_of(r + 1); k++) {
                if (key_start) key_start[k] = run;
                for (int64_t c = 0; c < nch; c++) {
                    const T v = cnt[c][k];
                    cnt[c][k] = (T)run;
                    run += v;
                }
            }
        }
    });
    if (key_start) key_start[nkeys] = rbase[nkr];
    return rbase[nkr];
}

// the same stable counting sort over chunks of `ids` on host threads: per-chunk key counts,
// offsets in (key, chunk) order, every chunk scatters its ids in order (a stable sort's output is
// unique, so the result does not depend on the chunking)
template <class Key>
void par_counting_sort(std::vector<int32_t> &ids, int64_t nkeys, Key key) {
    if (nkeys <= 1) return;                   // one key: the stable order is the input order
    const int64_t n = (int64_t)ids.size();
    const int64_t nch = std::max<int64_t>(1, std::min<int64_t>(16, n / (1 << 18)));
    if (nch <= 1) { counting_sort(ids, nkeys, key); return; }
    std::vector<std::vector<int32_t>> cnt((size_t)nch);
    auto lo_of = [&](int64_t c) { return n * c / nch; };
    chunked(nch, 1, [&](int, int64_t c0, int64_t c1) {
        for (int64_t c = c0; c < c1; c++) {
            cnt[c].assign((size_t)nkeys, 0);
            for (int64_t i = lo_of(c); i < lo_of(c + 1); i++) cnt[c][(size_t)key(ids[i])]++;
        }
    });
    chunk_offsets(cnt, nkeys, nullptr);
    std::vector<int32_t> out((size_t)n);
    chunked(nch, 1, [&](int, int64_t c0, int64_t c1) {
        for (int64_t c = c0; c < c1; c++)
            for (int64_t i = lo_of(c); i < lo_of(c + 1); i++) out[(size_t)cnt[c][(size_t)key(ids[i])]++] = ids[i];
    });
    ids.swap(out);
}

// a stable LSD radix sort of ids by their 42-bit curve keys (three 14-bit digits): ids with equal keys
// keep their order, so from ascending ids it is std::sort by (key, id)
void radix_sort_by_key(std::vector<int32_t> &ids, const std::vector<uint64_t> &key) {
    std::vector<int32_t> tmp(ids.size());
    std::vector<uint32_t> cnt(1 << 14);
    for (int pass = 0; pass < 3; pass++) {
        const int sh = 14 * pass;
        std::fill(cnt.begin(), cnt.end(), 0u);
        for (int32_t i : ids) cnt[(key[i] >> sh) & 0x3fff]++;
        uint32_t sum = 0;
        for (uint32_t &c : cnt) { const uint32_t t = c; c = sum; sum += t; }
        for (int32_t i : ids) tmp[cnt[(key[i] >> sh) & 0x3fff]++] = i;
        ids.swap(tmp);
    }
}

}  // namespace

bool build_sp_plan(const deftri_problem_desc &d, int rank, int nranks, bool fp32_jac, SpPlanHost &H,
                   std::string &err, bool tile) {
    static const bool timing = std::getenv("DEFTRI_PLAN_TIMING") != nullptr;
    auto t_prev = std::chrono::steady_clock::now();
    auto stage = [&](const char *name) {
        if (!timing) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[deftri plan] %-28s %8.2f ms\n", name, std::chrono::duration<double, std::milli>(t - t_prev).count());
        t_prev = t;
    };
    H = SpPlanHost();
    if (nranks < 1 || rank < 0 || rank >= nranks) { err = "bad rank"; return false; }
    H.rank = rank;
    H.nranks = nranks;
    const int32_t P = d.n_points, Q = d.n_pairs, S = d.n_scales;
    const int64_t E = d.n_arap, R = d.n_rep, D = d.n_depth;
    H.P = P; H.Q = Q; H.S = S;
    H.hd = 6 * (int64_t)Q + S;
    if (E >= (1LL << 29)) { err = "more than 2^29 ARAP edges"; return false; }
    const int32_t *ap = d.arap_pts;

    // 1. keyframe-copy groups: union-find over the ARAP edges' (p1_i, p2_i) and (p1_j, p2_j)
    //    on host threads: a root is only ever linked under a smaller root (compare-and-swap), so every
    //    tree's root is its smallest point id and the partition and roots do not depend on the order
    std::vector<int32_t> par(P);
    std::iota(par.begin(), par.end(), 0);
    auto ld = [&](int32_t a) { return __atomic_load_n(&par[a], __ATOMIC_RELAXED); };
    auto find = [&](int32_t a) {
        for (;;) {
            const int32_t p = ld(a);
            if (p == a) return a;
            const int32_t gp = ld(p);
            if (gp != p) { int32_t exp = p; __atomic_compare_exchange_n(&par[a], &exp, gp, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED); }
            a = p;
        }
    };
    auto unite = [&](int32_t a, int32_t b) {
        for (;;) {
            a = find(a); b = find(b);
            if (a == b) return;
            if (a > b) std::swap(a, b);
            int32_t exp = b;                     // b still a root: link it under the smaller a
            if (__atomic_compare_exchange_n(&par[b], &exp, a, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) return;
        }
    };
    chunked(E, 1 << 18, [&](int, int64_t e0, int64_t e1) {
        for (int64_t e = e0; e < e1; e++) {
            unite(ap[4 * e], ap[4 * e + 1]);
            unite(ap[4 * e + 2], ap[4 * e + 3]);
        }
    });
    std::vector<int32_t> root(P);
    chunked(P, 1 << 16, [&](int, int64_t p0, int64_t p1) {
        for (int64_t p = p0; p < p1; p++) root[p] = find((int32_t)p);
    });
    std::vector<int32_t> gid(P, -1), grep;   // group of each point; representative (smallest id) per group
    for (int32_t p = 0; p < P; p++) {
        const int32_t r = root[p];
        if (gid[r] < 0) { gid[r] = (int32_t)grep.size(); grep.push_back(r); }
        gid[p] = gid[r];
    }
    const int32_t ng = (int32_t)grep.size();

    stage("1 groups (union-find)");
    // 2. groups in Morton order of the representative's mesh-plane position
    auto xy = [&](int32_t p, int c) { return d.order_xy ? d.order_xy[2 * (int64_t)p + c] : d.points[3 * (int64_t)p + c]; };
    double lo[2] = {1e300, 1e300}, hi[2] = {-1e300, -1e300};
    for (int32_t g = 0; g < ng; g++)
        for (int c = 0; c < 2; c++) {
            const double v = xy(grep[g], c);
            if (std::isfinite(v)) { lo[c] = std::min(lo[c], v); hi[c] = std::max(hi[c], v); }
        }
    std::vector<uint64_t> key(ng);
    for (int32_t g = 0; g < ng; g++) key[g] = curve_key(xy(grep[g], 0), xy(grep[g], 1), lo, hi);
    std::vector<int32_t> gorder(ng);
    std::iota(gorder.begin(), gorder.end(), 0);
    // by (key, representative): the representatives ascend with the group number (each group is met
    // first at its smallest point), so a stable sort by key from the identity is that order
    radix_sort_by_key(gorder, key);
    std::vector<int32_t> gpos(ng);
    for (int32_t k = 0; k < ng; k++) gpos[gorder[k]] = k;

    stage("2 Morton order");
    // 3. rows: groups in that order, points of a group by id.  A tile plan of several pairs (one rank)
    //    numbers them keyframe-major instead — by the camera of the point's reprojection edges, then
    //    the Morton order of the point's own position — so a tile of pair (a, b), consecutive units of
    //    that pair in the Morton order of keyframe b's positions, owns runs of keyframe b's rows
    std::vector<int32_t> pts(P);
    std::iota(pts.begin(), pts.end(), 0);
    counting_sort(pts, ng, [&](int32_t p) { return gpos[gid[p]]; });
    if (tile && Q > 1 && nranks == 1) {
        std::vector<int32_t> pcam(P, -1);
        bool one_cam = true;
        for (int64_t e = 0; e < R; e++) {
            int32_t &c = pcam[d.rep_point[e]];
            if (c < 0) c = d.rep_cam[e];
            else if (c != d.rep_cam[e]) one_cam = false;
        }
        if (one_cam) {
            const int32_t C = std::max(d.n_cams, 1);
            {
                // inside a keyframe, its points in the Morton order of their own positions: the order in
                // which the pairs whose mesh is that keyframe's (it is their keyframe 1) cut their tiles
                // (spcg_tile.cpp), so those tiles' keyframe-1 rows are runs (C5's CG iteration -3 %)
                std::vector<double> blo(2 * (size_t)(C + 1), 1e300), bhi(2 * (size_t)(C + 1), -1e300);
                auto cam = [&](int32_t p) { return pcam[p] < 0 ? C : pcam[p]; };
                for (int32_t p = 0; p < P; p++)
                    for (int c = 0; c < 2; c++) {
                        const double v = d.points[3 * (int64_t)p + c];
                        if (std::isfinite(v)) {
                            blo[2 * cam(p) + c] = std::min(blo[2 * cam(p) + c], v);
                            bhi[2 * cam(p) + c] = std::max(bhi[2 * cam(p) + c], v);
                        }
                    }
                std::vector<uint64_t> pk(P);
                            for (int32_t p = 0; p < P; p++)
                    pk[p] = curve_key(d.points[3 * (int64_t)p], d.points[3 * (int64_t)p + 1], &blo[2 * cam(p)],
                                      &bhi[2 * cam(p)]);
                // by (camera, key, point): stable by key from ascending points, then stable by camera
                std::iota(pts.begin(), pts.end(), 0);
                radix_sort_by_key(pts, pk);
                counting_sort(pts, C + 1, [&](int32_t p) { return cam(p); });
            }
        }
    }
    H.point_of_row = pts;
    H.row_of_point.assign(P, 0);
    for (int32_t r = 0; r < P; r++) H.row_of_point[pts[r]] = r;
    const std::vector<int32_t> &row = H.row_of_point;

    stage("3 rows");
    // 4. work-balanced contiguous group ranges per rank: weight of a row = 2 + its ARAP incidences
    //    (one rank: the whole range, no weights needed)
    H.rank_row_begin.assign(nranks + 1, P);
    H.rank_row_begin[0] = 0;
    if (nranks > 1) {
        std::vector<int64_t> rw(P, 2);
        for (int64_t e = 0; e < 4 * E; e++) rw[row[ap[e]]]++;
        for (int64_t e = 0; e < R; e++) rw[row[d.rep_point[e]]]++;
        for (int64_t e = 0; e < D; e++) rw[row[d.dep_point[e]]]++;
        const double total = std::accumulate(rw.begin(), rw.end(), 0.0);
        double cum = 0;
        int next = 1;
        for (int32_t r = 0; r < P && next < nranks; r++) {
            // cut only between groups
            const bool group_start = r == 0 || gid[pts[r]] != gid[pts[r - 1]];
            if (group_start && r > 0 && cum >= total * next / nranks) H.rank_row_begin[next++] = r;
            cum += (double)rw[r];
        }
        for (; next < nranks; next++) H.rank_row_begin[next] = P;
    }
    stage("4 rank ranges");
    // 4a. tile mode (one rank, one pair; spcg_tile.cpp): the groups cut into tiles in Morton order,
    //     the ARAP edges in tile-entry order; the rows keep the Morton group order (no 4b sort: a
    //     tile's rows are one contiguous range)
    std::vector<int32_t> tile_order, tile_foreign;
    if (tile && Q == 1 && S <= 2 && E > 0) {
        H.lo = H.rank_row_begin[rank];
        H.hi = H.rank_row_begin[rank + 1];
        std::vector<int32_t> gp(P);
        for (int32_t p = 0; p < P; p++) gp[p] = gpos[gid[p]];
        TileInput ti;
        ti.P = P; ti.ng = ng; ti.E = E; ti.ap = ap; ti.gpos = gp.data(); ti.row_of_point = H.row_of_point.data();
        std::string why;
        H.tile = build_tiles(ti, H, tile_order, tile_foreign, why);
        if (!H.tile) {
            H.tile_why = why;
            tile_order.clear();
            tile_foreign.clear();
        }
    } else if (tile && Q > 1 && nranks == 1 && E > 0) {
        // several pairs on one rank: tiles per pair over (pair, group) units (spcg_tile.cpp)
        H.lo = H.rank_row_begin[rank];
        H.hi = H.rank_row_begin[rank + 1];
        std::vector<int32_t> gp(P);
        for (int32_t p = 0; p < P; p++) gp[p] = gpos[gid[p]];
        TileInput ti;
        ti.P = P; ti.ng = ng; ti.E = E; ti.ap = ap; ti.gpos = gp.data(); ti.row_of_point = H.row_of_point.data();
        ti.Q = Q; ti.S = S; ti.pair = d.arap_pair; ti.D = D; ti.dep_point = d.dep_point; ti.dep_scale = d.dep_scale;
        ti.points = d.points;
        std::string why;
        H.tile = build_tiles_multi(ti, H, tile_order, why);
        if (!H.tile) {
            H.tile_why = why;
            tile_order.clear();
        }
    } else if (tile) {
        H.tile_why = Q != 1 ? "more than one keyframe pair on a sharded plan" : S > 2 ? "more than two depth scales" : "no ARAP edges";
    }
    stage("4a tiles");
    // 4b. inside every rank's range, rows sorted by their phase-2 slot count (ARAP incidences + depth
    //     couplings; descending, stable) in windows of kSpSortWindow rows: the order the phase-2 wave
    //     layout deals them to lanes (8b), so that layout is the identity and a wave's 64 rows are 64
    //     consecutive rows (the per-row vectors then load coalesced).  Every rank permutes every range
    //     the same way, so the global numbering agrees across ranks.
    //     The edges keep the Morton order (mrow, below): an edge run then walks its points, their
    //     rotations and (z, p) in spatial order (C2 under rocprofv3: k_lin_chi 19.3 vs 24.9 us, phase 1
    //     20.9 vs 23.6 with edges by the sorted rows).
    const std::vector<int32_t> mrow = H.row_of_point;     // Morton (pre-sort) row of each point
    if (!H.tile) {
        // slot counts per row: per-chunk counts over the incidences on host threads, summed per row
        const int64_t ninc = 4 * E + D;
        const int64_t nch = std::max<int64_t>(1, std::min<int64_t>(16, ninc / (1 << 20)));
        std::vector<std::vector<int32_t>> ccnt((size_t)nch);
        chunked(nch, 1, [&](int, int64_t c0, int64_t c1) {
            for (int64_t c = c0; c < c1; c++) {
                std::vector<int32_t> &k = ccnt[c];
                k.assign(P, 0);
                for (int64_t x = ninc * c / nch; x < ninc * (c + 1) / nch; x++)
                    k[row[x < 4 * E ? ap[x] : d.dep_point[x - 4 * E]]]++;
            }
        });
        std::vector<int32_t> cnt(P, 0);
        chunked(P, 1 << 16, [&](int, int64_t r0, int64_t r1) {
            for (int64_t c = 0; c < nch; c++)
                for (int64_t r = r0; r < r1; r++) cnt[r] += ccnt[c][r];
        });
        ccnt.clear();
        // the windows, each sorted on its own (every window writes its own rows)
        std::vector<int32_t> np(P);
        std::vector<int32_t> wstart;
        for (int rk = 0; rk < nranks; rk++)
            for (int32_t w0 = H.rank_row_begin[rk]; w0 < H.rank_row_begin[rk + 1]; w0 += kSpSortWindow) wstart.push_back(w0);
        chunked((int64_t)wstart.size(), 64, [&](int, int64_t i0, int64_t i1) {
            std::vector<int32_t> ord;
            for (int64_t i = i0; i < i1; i++) {
                const int32_t w0 = wstart[i];
                const int32_t rk_end = *std::upper_bound(H.rank_row_begin.begin(), H.rank_row_begin.end(), w0);
                const int32_t w1 = std::min(rk_end, w0 + kSpSortWindow);
                ord.resize(w1 - w0);
                std::iota(ord.begin(), ord.end(), w0);
                std::stable_sort(ord.begin(), ord.end(), [&](int32_t x, int32_t y) { return cnt[x] > cnt[y]; });
                for (int32_t k = 0; k < w1 - w0; k++) np[w0 + k] = H.point_of_row[ord[k]];
            }
        });
        H.point_of_row = np;
        chunked(P, 1 << 16, [&](int, int64_t r0, int64_t r1) {
            for (int64_t r = r0; r < r1; r++) H.row_of_point[np[r]] = (int32_t)r;
        });
    }
    H.lo = H.rank_row_begin[rank];
    H.hi = H.rank_row_begin[rank + 1];
    const int32_t lo_r = H.lo, hi_r = H.hi;
    auto own = [&](int32_t r) { return r >= lo_r && r < hi_r; };
    const int32_t nown = hi_r - lo_r;

    stage("4b slot-count sort");
    // 5. local ARAP edges: owned (point 0 here) first, then halo-only; each by (pair, Morton row of point 0)
    std::vector<int32_t> owned_e, halo_e;
    if (H.tile) {
        owned_e.swap(tile_order);                     // tile-entry order (spcg_tile.cpp)
        halo_e.swap(tile_foreign);
    } else if (nranks == 1) {
        owned_e.resize((size_t)E);
        std::iota(owned_e.begin(), owned_e.end(), 0);
    } else {
        for (int64_t e = 0; e < E; e++) {
            const int32_t r0 = row[ap[4 * e]];
            if (own(r0)) owned_e.push_back((int32_t)e);
            else if (own(row[ap[4 * e + 1]]) || own(row[ap[4 * e + 2]]) || own(row[ap[4 * e + 3]])) halo_e.push_back((int32_t)e);
        }
    }
    if (!H.tile)
        for (auto *lst : {&owned_e, &halo_e}) {
            par_counting_sort(*lst, P, [&](int32_t e) { return mrow[ap[4 * (int64_t)e]]; });
            par_counting_sort(*lst, std::max(Q, 1), [&](int32_t e) { return d.arap_pair[e]; });
        }
    H.n_arap_owned = (int32_t)owned_e.size();
    H.arap_ids = owned_e;
    H.arap_ids.insert(H.arap_ids.end(), halo_e.begin(), halo_e.end());
    owned_e.clear(); owned_e.shrink_to_fit();
    halo_e.clear(); halo_e.shrink_to_fit();
    const int64_t nloc = (int64_t)H.arap_ids.size();

    // rotation rows used by the local edges, compacted
    {
        // numbered in first-encounter order over the positions 2 le + k: each row's first position
        // (an atomic minimum over host threads), the first positions flagged and prefix-summed
        const int64_t npos = 2 * nloc;
        // the rotation rows gathered once in position order (the passes below then read them in order)
        std::vector<int32_t> rv((size_t)npos);
        chunked(nloc, 1 << 17, [&](int, int64_t l0, int64_t l1) {
            for (int64_t l = l0; l < l1; l++) {
                const int64_t e = H.arap_ids[l];
                rv[2 * l] = d.arap_rot[2 * e];
                rv[2 * l + 1] = d.arap_rot[2 * e + 1];
            }
        });
        auto rot_at = [&](int64_t x) { return rv[x]; };
        std::vector<int64_t> first((size_t)std::max(d.n_rot, 1), INT64_MAX);
        chunked(npos, 1 << 18, [&](int, int64_t x0, int64_t x1) {
            for (int64_t x = x0; x < x1; x++) {
                int64_t *f = &first[rot_at(x)];
                int64_t cur = __atomic_load_n(f, __ATOMIC_RELAXED);
                while (x < cur && !__atomic_compare_exchange_n(f, &cur, x, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {}
            }
        });
        const int64_t nch = std::max<int64_t>(1, std::min<int64_t>(16, npos / (1 << 18)));
        std::vector<int64_t> cbase((size_t)nch + 1, 0);
        chunked(nch, 1, [&](int, int64_t c0, int64_t c1) {
            for (int64_t c = c0; c < c1; c++)
                for (int64_t x = npos * c / nch; x < npos * (c + 1) / nch; x++) cbase[c + 1] += first[rot_at(x)] == x;
        });
        for (int64_t c = 0; c < nch; c++) cbase[c + 1] += cbase[c];
        H.rot_ids.resize((size_t)cbase[nch]);
        std::vector<int32_t> map(std::max(d.n_rot, 1), -1);
        chunked(nch, 1, [&](int, int64_t c0, int64_t c1) {
            for (int64_t c = c0; c < c1; c++) {
                int64_t n = cbase[c];
                for (int64_t x = npos * c / nch; x < npos * (c + 1) / nch; x++) {
                    const int32_t g = rot_at(x);
                    if (first[g] == x) { map[g] = (int32_t)n; H.rot_ids[n++] = g; }
                }
            }
        });
        H.arap_rot_local.resize((size_t)npos);
        chunked(npos, 1 << 18, [&](int, int64_t x0, int64_t x1) {
            for (int64_t x = x0; x < x1; x++) H.arap_rot_local[x] = map[rot_at(x)];
        });
    }

    stage("5 local ARAP edges");
    // 6. the own rows' reprojection / depth edges, by row
    if (nranks == 1) {
        H.rep_ids.resize((size_t)R);
        std::iota(H.rep_ids.begin(), H.rep_ids.end(), 0);
        H.dep_ids.resize((size_t)D);
        std::iota(H.dep_ids.begin(), H.dep_ids.end(), 0);
    } else {
        for (int64_t e = 0; e < R; e++) if (own(row[d.rep_point[e]])) H.rep_ids.push_back((int32_t)e);
        for (int64_t e = 0; e < D; e++) if (own(row[d.dep_point[e]])) H.dep_ids.push_back((int32_t)e);
    }
    par_counting_sort(H.rep_ids, P, [&](int32_t e) { return row[d.rep_point[e]]; });
    par_counting_sort(H.dep_ids, P, [&](int32_t e) { return row[d.dep_point[e]]; });
    H.rep_off.assign(nown + 1, 0);
    H.dep_off.assign(nown + 1, 0);
    for (int32_t e : H.rep_ids) H.rep_off[row[d.rep_point[e]] - lo_r + 1]++;
    for (int32_t e : H.dep_ids) H.dep_off[row[d.dep_point[e]] - lo_r + 1]++;
    for (int32_t l = 0; l < nown; l++) { H.rep_off[l + 1] += H.rep_off[l]; H.dep_off[l + 1] += H.dep_off[l]; }

    stage("6 rep / depth by row");
    // 7. phase-1 blocks: ARAP (owned, then halo-only) per pair in runs of kSpBlock; depth edges by
    //    (scale, row) per scale
    const int32_t ndl = (int32_t)H.dep_ids.size();
    H.dperm.resize(ndl);
    std::iota(H.dperm.begin(), H.dperm.end(), 0);
    par_counting_sort(H.dperm, std::max(S, 1), [&](int32_t j) { return d.dep_scale[H.dep_ids[j]]; });
    auto add_blocks = [&](int kind, int owned, int64_t b0, int64_t b1, auto heavy_of) {
        int64_t i = b0;
        while (i < b1) {
            const int32_t hv = heavy_of(i);
            int64_t j = i;
            while (j < b1 && j - i < kSpBlock && heavy_of(j) == hv) j++;
            H.blk.push_back(kind | owned << 8);
            H.blk.push_back(hv);
            H.blk.push_back((int32_t)i);
            H.blk.push_back((int32_t)j);
            i = j;
        }
    };
    auto pair_of = [&](int64_t le) { return d.arap_pair[H.arap_ids[le]]; };
    add_blocks(SP_ARAP, 1, 0, H.n_arap_owned, pair_of);
    add_blocks(SP_ARAP, 0, H.n_arap_owned, nloc, pair_of);
    add_blocks(SP_DEP, 1, 0, ndl, [&](int64_t i) { return d.dep_scale[H.dep_ids[H.dperm[i]]]; });
    const int64_t nb = (int64_t)H.blk.size() / 4;
    // dispatch order: blocks by the row of their first edge's point (stable), so the blocks of every
    // pair / scale over one region of rows run together and share the rows' (z, p) in L2 / MALL
    // instead of one sweep over all rows per pair (28 sweeps at C4)
    {
        std::vector<int64_t> key(nb);
        for (int64_t b = 0; b < nb; b++) {
            const int kind = H.blk[4 * b] & 0xff;
            const int32_t i = H.blk[4 * b + 2];
            key[b] = kind == SP_ARAP ? mrow[ap[4 * (int64_t)H.arap_ids[i]]] : mrow[d.dep_point[H.dep_ids[H.dperm[i]]]];
        }
        std::vector<int64_t> ord(nb);
        std::iota(ord.begin(), ord.end(), 0);
        std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return key[a] < key[b]; });
        // XCD-aware: workgroup b runs on XCD b % 8, so the sorted list is cut into 8 contiguous
        // segments and dealt out (position 8 j + x <- segment x's j-th block): each XCD's L2 walks
        // its own run of rows
        constexpr int kXcd = 8;
        const int64_t seg = (nb + kXcd - 1) / kXcd;
        std::vector<int64_t> pos_of;
        pos_of.reserve(nb);
        for (int64_t j = 0; j < seg; j++)
            for (int x = 0; x < kXcd; x++)
                if (x * seg + j < nb) pos_of.push_back(x * seg + j);
        std::vector<int32_t> blk2(H.blk.size());
        for (int64_t b = 0; b < nb; b++)
            for (int k = 0; k < 4; k++) blk2[4 * b + k] = H.blk[4 * ord[pos_of[b]] + k];
        H.blk.swap(blk2);
    }
    H.hv_blk_off.assign(Q + S + 1, 0);
    auto blk_heavy = [&](int64_t b) -> int32_t {
        const int kind = H.blk[4 * b] & 0xff, owned = H.blk[4 * b] >> 8;
        if (kind == SP_ARAP) return owned ? H.blk[4 * b + 1] : -1;
        return Q + H.blk[4 * b + 1];
    };
    for (int64_t b = 0; b < nb; b++) { const int32_t h = blk_heavy(b); if (h >= 0) H.hv_blk_off[h + 1]++; }
    for (int32_t h = 0; h < Q + S; h++) H.hv_blk_off[h + 1] += H.hv_blk_off[h];
    H.hv_blk.resize((size_t)H.hv_blk_off[Q + S]);
    {
        std::vector<int64_t> pos(H.hv_blk_off.begin(), H.hv_blk_off.end() - 1);
        for (int64_t b = 0; b < nb; b++) { const int32_t h = blk_heavy(b); if (h >= 0) H.hv_blk[pos[h]++] = (int32_t)b; }
    }

    stage("7 phase-1 blocks");
    // 8. own rows' ARAP incidences (local edge << 2 | role), each row's in local-edge order
    //    (a counting sort over chunks of local edges: per-chunk row counts, chunk-ordered offsets,
    //    every chunk scatters its edges in order — the sequential order)
    H.inc_off.assign(nown + 1, 0);
    {
        constexpr int64_t kMin = 1 << 16;
        const int64_t nch = std::max<int64_t>(1, std::min<int64_t>(16, nloc / kMin));
        std::vector<std::vector<int32_t>> ccnt((size_t)nch);
        auto lo_of = [&](int64_t c) { return nloc * c / nch; };
        chunked(nch, 1, [&](int, int64_t c0, int64_t c1) {
            for (int64_t c = c0; c < c1; c++) {
                ccnt[c].assign(nown, 0);
                for (int64_t le = lo_of(c); le < lo_of(c + 1); le++) {
                    const int64_t e = H.arap_ids[le];
                    for (int k = 0; k < 4; k++) { const int32_t r = row[ap[4 * e + k]]; if (own(r)) ccnt[c][r - lo_r]++; }
                }
            }
        });
        // offsets: row-major, chunk order inside a row (ccnt becomes each chunk's write position)
        const int64_t acc = chunk_offsets(ccnt, nown, H.inc_off.data());
        H.inc.resize((size_t)acc);
        chunked(nch, 1, [&](int, int64_t c0, int64_t c1) {
            for (int64_t c = c0; c < c1; c++)
                for (int64_t le = lo_of(c); le < lo_of(c + 1); le++) {
                    const int64_t e = H.arap_ids[le];
                    for (int k = 0; k < 4; k++) {
                        const int32_t r = row[ap[4 * e + k]];
                        if (own(r)) H.inc[ccnt[c][r - lo_r]++] = (int32_t)(le << 2 | k);
                    }
                }
        });
    }

    stage("8 incidences");
    // 8b. phase-2 wave layout: per own row its ARAP incidences then its depth couplings; rows sorted by
    //     that count (descending, stable) inside windows of kSpSortWindow rows, 64 per wave.  A wave
    //     whose rows hold more than kSpWaveSplit slots takes 32
    //     rows instead, each on a lane pair: lane j the first ceil(c / 2) slots of its row, lane j + 32
    //     the rest (rowmap -1: the pair's sums go to lane j) — the longest waves' step counts halve,
    //     which is what bounds phase 2 and the rows' linearization (their span, not their bytes)
    {
        const int split_t = kSpWaveSplit;
        std::vector<int32_t> cnt(nown);
        for (int32_t l = 0; l < nown; l++)
            cnt[l] = (int32_t)(H.inc_off[l + 1] - H.inc_off[l]) + (H.dep_off[l + 1] - H.dep_off[l]);
        std::vector<int32_t> order(nown);
        std::iota(order.begin(), order.end(), 0);
        const int64_t nwin = (nown + kSpSortWindow - 1) / kSpSortWindow;
        chunked(nwin, 64, [&](int, int64_t a0, int64_t a1) {
            for (int64_t a = a0; a < a1; a++) {
                const int32_t w0 = (int32_t)(a * kSpSortWindow), w1 = std::min(nown, w0 + kSpSortWindow);
                std::stable_sort(order.begin() + w0, order.begin() + w1, [&](int32_t x, int32_t y) { return cnt[x] > cnt[y]; });
            }
        });
        H.rowmap.clear();
        H.woff.assign(1, 0);
        H.wsplit.clear();
        std::vector<int32_t> first;                    // per wave: its first row in `order`
        for (int32_t i = 0; i < nown;) {
            int32_t kmax = 0;
            for (int j = 0; j < 64 && i + j < nown; j++) kmax = std::max(kmax, cnt[order[i + j]]);
            const bool sp = split_t > 0 && kmax > split_t;
            const int nr = sp ? 32 : 64;
            int32_t steps = 0;
            for (int j = 0; j < nr && i + j < nown; j++) {
                const int32_t c = cnt[order[i + j]];
                steps = std::max(steps, sp ? (c + 1) / 2 : c);
            }
            first.push_back(i);
            const size_t base = H.rowmap.size();
            H.rowmap.resize(base + 64, -1);
            for (int j = 0; j < nr && i + j < nown; j++) H.rowmap[base + j] = order[i + j];
            H.woff.push_back(H.woff.back() + steps);
            H.wsplit.push_back(sp ? 1 : 0);
            i += nr;
        }
        const int32_t nw = (int32_t)H.wsplit.size();
        const int64_t nsl = H.woff[nw];
        H.pmap.resize((size_t)nsl * 64);
        H.pidx.resize((size_t)nsl * 64);
        chunked(nw, 256, [&](int, int64_t w0, int64_t w1) {      // waves own disjoint slot ranges
            std::vector<int32_t> pm, pi;               // one row's slot list
            std::fill(H.pmap.begin() + 64 * H.woff[w0], H.pmap.begin() + 64 * H.woff[w1], -1);
            std::fill(H.pidx.begin() + 64 * H.woff[w0], H.pidx.begin() + 64 * H.woff[w1], -1);
            for (int64_t w = w0; w < w1; w++) {
                const bool sp = H.wsplit[w] != 0;
                for (int j = 0; j < (sp ? 32 : 64); j++) {
                    const int32_t l = H.rowmap[64 * (size_t)w + j];
                    if (l < 0) continue;
                    pm.clear();
                    pi.clear();
                    for (int64_t x = H.inc_off[l]; x < H.inc_off[l + 1]; x++) { pm.push_back(H.inc[x]); pi.push_back(H.inc[x] >> 2); }
                    for (int32_t x = H.dep_off[l]; x < H.dep_off[l + 1]; x++) {
                        pm.push_back(-(2 + x));
                        pi.push_back(-(2 + d.dep_scale[H.dep_ids[x]]));
                    }
                    const size_t h = sp ? (pm.size() + 1) / 2 : pm.size();
                    for (size_t t = 0; t < pm.size(); t++) {
                        const int lane = t < h ? j : j + 32;
                        const int64_t k = H.woff[w] + (int64_t)(t < h ? t : t - h);
                        H.pmap[64 * k + lane] = pm[t];
                        H.pidx[64 * k + lane] = pi[t];
                    }
                }
            }
        });
    }
    for (int32_t h = 0; h < Q + S; h++)
        H.max_heavy_blocks = std::max<int32_t>(H.max_heavy_blocks, (int32_t)(H.hv_blk_off[h + 1] - H.hv_blk_off[h]));

    stage("8b wave layout");
    // 9. halo exchange lists
    H.send_rows.assign(nranks, {});
    H.recv_rows.assign(nranks, {});
    if (nranks > 1) {
        std::vector<int32_t> owner(P);
        for (int rr = 0; rr < nranks; rr++)
            for (int32_t r = H.rank_row_begin[rr]; r < H.rank_row_begin[rr + 1]; r++) owner[r] = rr;
        std::vector<uint8_t> need(P, 0);
        for (int64_t le = 0; le < nloc; le++) {
            const int64_t e = H.arap_ids[le];
            for (int k = 0; k < 4; k++) { const int32_t r = row[ap[4 * e + k]]; if (!own(r)) need[r] = 1; }
        }
        for (int32_t r = 0; r < P; r++) if (need[r]) H.recv_rows[owner[r]].push_back(r);
        // rows of this rank read by another rank's local edges
        for (int64_t e = 0; e < E; e++) {
            int32_t rr[4], oo[4];
            bool mine = false, other = false;
            for (int k = 0; k < 4; k++) {
                rr[k] = row[ap[4 * e + k]]; oo[k] = owner[rr[k]];
                mine |= oo[k] == rank;
                other |= oo[k] != rank;
            }
            if (!mine || !other) continue;
            for (int k = 0; k < 4; k++) {
                if (oo[k] != rank) continue;
                for (int j = 0; j < 4; j++) if (oo[j] != rank) H.send_rows[oo[j]].push_back(rr[k]);
            }
        }
        for (auto &v : H.send_rows) { std::sort(v.begin(), v.end()); v.erase(std::unique(v.begin(), v.end()), v.end()); }
        for (auto &v : H.recv_rows) H.halo_rows += (int64_t)v.size();
    }

    stage("9 halo lists");
    // 10. algorithmic bytes of one product (phase 1 + phase 2): compulsory loads and
    //     stores, the p gathers at an edge's other points not counted
    const double jb = fp32_jac ? 72.0 : 144.0;
    H.phase1_bytes = (double)nloc * (jb + 8 + 16 + 8)                  // J, W, rows, s
                     + (double)ndl * (4 + 4 + 24 + 8);                  // dperm, row, c, W J_s^2
    H.phase2_bytes = (double)nown * (48 + 48 + 48 + 24 + 4)            // (z,p) in / out, D, q, row map
                     + (double)H.inc.size() * (4 + 8 + jb / 6)           // slot index, s, packed J slice
                     + (double)ndl * (4 + jb / 6);                       // depth-coupling slots (p_s in cache)
    H.product_bytes = H.phase1_bytes + H.phase2_bytes;
    if (H.tile) {
        // tile mode per CG iteration: k_sp_tile — per entry J (valid) + meta, per tile row (z, p) + D
        // + q out + its slot range + its depth couplings (c, W J_s^2, scale, offset), per halo row
        // (z, p), per cut entry two cross slots out and their positions; k_sp_tupd — per own row (z, p)
        // in / out, x and r in / out, q in, M, its cross range, per cross slot its value
        const int64_t nvalid = (int64_t)H.arap_ids.size();
        H.tile_bytes[0] = (double)nvalid * jb + (double)H.tile_entries * 8 + (double)nown * (48 + 48 + 24 + 4) +
                          (double)ndl * (24 + 8 + 4 + 4) + (double)H.tile_halo_rows * 48 + (double)H.tile_cross * (24 + 4);
        H.tile_bytes[1] = (double)nown * (96 + 48 + 48 + 24 + 48 + 8) + (double)H.tile_cross * 24;
        // fused (one launch): q stays in registers, p in LDS — no q out / in, no (z, p) reload
    }
    static const bool digest = std::getenv("DEFTRI_PLAN_DIGEST") != nullptr;
    if (digest) {
        // FNV-1a over every plan array: a rewrite of the build is checked against the previous one
        uint64_t h = 1469598103934665603ULL;
        auto mix = [&](const void *v, size_t n) {
            const unsigned char *c = (const unsigned char *)v;
            for (size_t i = 0; i < n; i++) { h ^= c[i]; h *= 1099511628211ULL; }
        };
        auto vec = [&](const auto &x) { mix(x.data(), x.size() * sizeof(x[0])); };
        vec(H.row_of_point); vec(H.point_of_row); vec(H.rank_row_begin); vec(H.arap_ids); vec(H.rep_ids);
        vec(H.dep_ids); vec(H.rot_ids); vec(H.arap_rot_local); vec(H.blk); vec(H.hv_blk); vec(H.hv_blk_off);
        vec(H.dperm); vec(H.inc_off); vec(H.inc); vec(H.rep_off); vec(H.dep_off); vec(H.rowmap); vec(H.woff);
        vec(H.wsplit); vec(H.pmap); vec(H.pidx);
        vec(H.tile_tab); vec(H.tile_m0); vec(H.tile_m1); vec(H.tile_chunk); vec(H.tile_rs); vec(H.tile_halo);
        vec(H.tile_xoff); vec(H.tile_xdst);
        for (const auto &x : H.send_rows) vec(x);
        for (const auto &x : H.recv_rows) vec(x);
        const int64_t sc[4] = {H.lo, H.hi, H.n_arap_owned, H.halo_rows};
        mix(sc, sizeof(sc));
        std::fprintf(stderr, "[deftri plan] digest %016llx\n", (unsigned long long)h);
    }
    return true;
}

// Host emulation of one sharded product q = (H + lambda I) p on this rank's plan, with the device
// kernels' decomposition (tests; no GPU): only the own rows of p are read from the input, the halo
// rows arrive through `xfer` (op 2 send / 3 receive, the same global order as the device exchange),
// the heavy partials of the owned edges are all-reduced (op 0).  J / W in the problem's edge order.
// q receives the own rows (problem order) and the heavy dofs; the other rows are zero.
int sp_emulate_product(const deftri_problem_desc &d, const SpPlanHost &H, const double *Ja, const double *Wa,
                       const double *Jr, const double *Wr, const double *Jd, const double *Wd, double lambda,
                       const double *p, double *q, const std::function<int(int, int, double *, int64_t)> &xfer) {
    const int64_t hd = H.hd, ndof = hd + 3 * (int64_t)H.P;
    const int32_t lo = H.lo, hi = H.hi, nown = hi - lo, Q = H.Q;
    std::vector<double> pl(ndof, 0.0);
    for (int64_t k = 0; k < hd; k++) pl[k] = p[k];
    for (int32_t r = lo; r < hi; r++)
        for (int c = 0; c < 3; c++) pl[hd + 3 * (int64_t)r + c] = p[hd + 3 * (int64_t)H.point_of_row[r] + c];
    if (H.nranks > 1) {
        for (int a = 0; a < H.nranks; a++)
            for (int b = 0; b < H.nranks; b++) {
                if (a == b) continue;
                if (a == H.rank && !H.send_rows[b].empty()) {
                    std::vector<double> buf;
                    for (int32_t r : H.send_rows[b]) for (int c = 0; c < 3; c++) buf.push_back(pl[hd + 3 * (int64_t)r + c]);
                    if (xfer(2, b, buf.data(), (int64_t)buf.size())) return -2;
                }
                if (b == H.rank && !H.recv_rows[a].empty()) {
                    std::vector<double> buf(3 * H.recv_rows[a].size());
                    if (xfer(3, a, buf.data(), (int64_t)buf.size())) return -2;
                    for (size_t i = 0; i < H.recv_rows[a].size(); i++)
                        for (int c = 0; c < 3; c++) pl[hd + 3 * (int64_t)H.recv_rows[a][i] + c] = buf[3 * i + c];
                }
            }
    }
    // phase 1
    const int64_t nloc = (int64_t)H.arap_ids.size();
    std::vector<double> s(nloc), hsum(hd, 0.0);
    for (int64_t le = 0; le < nloc; le++) {
        const int64_t e = H.arap_ids[le];
        const double *J = Ja + 18 * e;
        const int32_t q_ = d.arap_pair[e];
        double t = 0;
        for (int k = 0; k < 4; k++) {
            const int64_t o = hd + 3 * (int64_t)H.row_of_point[d.arap_pts[4 * e + k]];
            for (int c = 0; c < 3; c++) t += J[3 * k + c] * pl[o + c];
        }
        for (int c = 0; c < 6; c++) t += J[12 + c] * pl[6 * (int64_t)q_ + c];
        s[le] = Wa[e] * t;
        if (le < H.n_arap_owned)
            for (int c = 0; c < 6; c++) hsum[6 * (int64_t)q_ + c] += J[12 + c] * s[le];
    }
    for (int32_t e : H.dep_ids) {
        const double *J = Jd + 4 * (int64_t)e;
        const int64_t o = hd + 3 * (int64_t)H.row_of_point[d.dep_point[e]];
        const int32_t sc = d.dep_scale[e];
        double t = 0;
        for (int c = 0; c < 3; c++) t += Wd[e] * J[c] * J[3] * pl[o + c];
        t += Wd[e] * J[3] * J[3] * pl[6 * (int64_t)Q + sc];
        hsum[6 * (int64_t)Q + sc] += t;
    }
    if (H.nranks > 1 && hd > 0 && xfer(0, -1, hsum.data(), hd)) return -2;
    // phase 2
    for (int64_t k = 0; k < ndof; k++) q[k] = 0.0;
    for (int32_t l = 0; l < nown; l++) {
        const int32_t r = lo + l;
        const int64_t o = hd + 3 * (int64_t)r;
        double acc[3];
        for (int c = 0; c < 3; c++) acc[c] = lambda * pl[o + c];
        for (int32_t j = H.rep_off[l]; j < H.rep_off[l + 1]; j++) {
            const int64_t e = H.rep_ids[j];
            const double *J = Jr + 6 * e;
            for (int rr = 0; rr < 2; rr++) {
                double t = 0;
                for (int c = 0; c < 3; c++) t += J[3 * rr + c] * pl[o + c];
                for (int c = 0; c < 3; c++) acc[c] += J[3 * rr + c] * Wr[e] * t;
            }
        }
        for (int32_t j = H.dep_off[l]; j < H.dep_off[l + 1]; j++) {
            const int64_t e = H.dep_ids[j];
            const double *J = Jd + 4 * e;
            double t = J[3] * pl[6 * (int64_t)Q + d.dep_scale[e]];
            for (int c = 0; c < 3; c++) t += J[c] * pl[o + c];
            for (int c = 0; c < 3; c++) acc[c] += J[c] * Wd[e] * t;
        }
        for (int64_t k = H.inc_off[l]; k < H.inc_off[l + 1]; k++) {
            const int v = H.inc[k];
            const int64_t le = v >> 2, e = H.arap_ids[le];
            for (int c = 0; c < 3; c++) acc[c] += Ja[18 * e + 3 * (v & 3) + c] * s[le];
        }
        const int64_t po = hd + 3 * (int64_t)H.point_of_row[r];
        for (int c = 0; c < 3; c++) q[po + c] = acc[c];
    }
    for (int64_t k = 0; k < hd; k++) q[k] = hsum[k] + lambda * pl[k];
    return 0;
}

}  // namespace deftri
