// spcg_tile.cpp — the tile layout of the iterative plan's fused product (spcg.h "tile mode").
//
// One rank, one keyframe pair (the two-view graphs of BASELINE C2 and the 500k north-star size,
// g2oBundleAdjustment.cc:640-953 with one pair): the product q = (H + lambda I) p is formed by ONE
// edge pass in which every ARAP edge is read once.  The mesh vertices' keyframe-copy groups (2 rows
// each: p1_i, p2_i) are cut, in Morton order, into tiles of consecutive groups; a tile is one
// workgroup.  An edge (p1_i, p2_i, p1_j, p2_j, T_g) belongs to the tile of its vertex i ("out-edge");
// its contribution J_{p1_i}^T s, J_{p2_i}^T s to the own rows is summed over the edges of the same
// vertex (consecutive lanes, a segmented wave scan), its contribution to the rows of j goes to an LDS
// slot of j's row when j is in the tile, else to a cross slot in HBM that the update launch adds
// ("cut" edge).  So s_e never leaves the workgroup and J is read once — where the two-phase chain read
// J in phase 1, stored s_e and read J again (packed per slot) in phase 2.
//
// Layout (per tile, 64-entry chunks = one wave per round):
//   entries  the tile's out-edges grouped by vertex (unit), vertices in Morton order; a unit never
//            straddles a chunk (the chunk is padded instead); local edge le = the order of the valid
//            entries (so J, W, E, chi of the edges are in entry order: the loads of a chunk coalesce)
//   meta     2 words per entry (spcg.h kTm*): word0 = the LDS rows of p1_j, p2_j (12 bits each) and
//            the flags (segment head / last, swap: p1_i is the group's second row, valid, cut);
//            word1 = the LDS remote slots of p1_j, p2_j (12 bits each) and the unit's first row (8)
//   chunk    per 64 entries: the le of its first valid entry, its first cross slot
//   rows     the tile's own rows (consecutive), then its halo rows (rows of cut edges' j vertices)
//   slots    per own row its incoming LDS contributions, contiguous (row r: trs[r] = begin | count << 16)
//   cross    per own row (all tiles) the cross slots aimed at it, contiguous in source order (xoff);
//            per cut entry its two slots' positions (xdst)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <numeric>
#include <string>
#include <vector>

#include "host_threads.h"
#include "spcg.h"

namespace deftri {

// DEFTRI_PLAN_TIMING: the tiles' shapes (rows, halo rows, entries, slots; the cross slots)
static void tile_shape_stats(const std::vector<int32_t> &tab, int32_t nt, int64_t nx) {
    if (nt <= 0) return;
    for (int f = 1; f <= 6; f++) {
        if (f == 3 || f == 5) continue;
        std::vector<int32_t> v(nt);
        for (int32_t t = 0; t < nt; t++) v[t] = tab[8 * (size_t)t + f];
        std::sort(v.begin(), v.end());
        double s = 0;
        for (int32_t x : v) s += x;
        std::fprintf(stderr, "[deftri plan]   4a tiles %d, %-6s min %d mean %.1f p50 %d p90 %d max %d\n", nt,
                     f == 1 ? "rows" : f == 2 ? "halo" : f == 4 ? "ne" : "slots", v[0], s / nt, v[nt / 2],
                     v[(size_t)(0.9 * nt)], v[nt - 1]);
    }
    std::fprintf(stderr, "[deftri plan]   4a cross slots %lld\n", (long long)nx);
}

// The entries stage on host threads: each thread builds a contiguous range of tiles into buffers of
// its own, its counters starting from zero; the buffers are then concatenated in tile order and the
// earlier ranges' sizes added to the tile table's entry and halo bases, the chunk bases and the cross
// slot ids — the arrays one sequential pass over the tiles writes (plan digests unchanged)
namespace {

constexpr int32_t kLeForeign = 1 << 30;                 // a chunk base counted among the halo-only edges

struct TileBuf {
    int64_t t0 = 0, t1 = 0;
    std::vector<uint32_t> m0, m1;
    std::vector<int32_t> halo, order, foreign, chunk;   // chunk: (le, first cross slot) per 64 entries
    std::vector<std::pair<int32_t, int32_t>> xt;        // (target row, cross slot)
    int64_t nx = 0;
    int32_t segmax = 1, max_lds = 0;
    const char *err = nullptr;
};

bool merge_tile_bufs(std::vector<TileBuf> &B, int nb, SpPlanHost &H, std::vector<int32_t> &order,
                     std::vector<int32_t> *order_foreign, int64_t n_owned, std::vector<std::pair<int32_t, int32_t>> &xt,
                     int64_t &nx, int32_t &segmax, int32_t &max_lds, std::string &why) {
    for (int b = 0; b < nb; b++)
        if (B[b].err) { why = B[b].err; return false; }
    std::vector<int64_t> bm(nb + 1, 0), bh(nb + 1, 0), bo(nb + 1, 0), bf(nb + 1, 0), bc(nb + 1, 0), bx(nb + 1, 0),
        bt(nb + 1, 0);
    for (int b = 0; b < nb; b++) {
        bm[b + 1] = bm[b] + (int64_t)B[b].m0.size();
        bh[b + 1] = bh[b] + (int64_t)B[b].halo.size();
        bo[b + 1] = bo[b] + (int64_t)B[b].order.size();
        bf[b + 1] = bf[b] + (int64_t)B[b].foreign.size();
        bc[b + 1] = bc[b] + (int64_t)B[b].chunk.size();
        bx[b + 1] = bx[b] + B[b].nx;
        bt[b + 1] = bt[b] + (int64_t)B[b].xt.size();
        segmax = std::max(segmax, B[b].segmax);
        max_lds = std::max(max_lds, B[b].max_lds);
    }
    if (bm[nb] >= (1LL << 31) || bx[nb] >= (1LL << 31)) { why = "more than 2^31 tile entries or cross slots"; return false; }
    H.tile_m0.resize(bm[nb]);
    H.tile_m1.resize(bm[nb]);
    H.tile_halo.resize(bh[nb]);
    H.tile_chunk.resize(bc[nb]);
    order.resize(bo[nb]);
    if (order_foreign) order_foreign->resize(bf[nb]);
    xt.resize(bt[nb]);
    auto cp = [&](int, int64_t b0, int64_t b1) {
        for (int64_t b = b0; b < b1; b++) {
            TileBuf &X = B[b];
            std::copy(X.m0.begin(), X.m0.end(), H.tile_m0.begin() + bm[b]);
            std::copy(X.m1.begin(), X.m1.end(), H.tile_m1.begin() + bm[b]);
            std::copy(X.halo.begin(), X.halo.end(), H.tile_halo.begin() + bh[b]);
            std::copy(X.order.begin(), X.order.end(), order.begin() + bo[b]);
            if (order_foreign) std::copy(X.foreign.begin(), X.foreign.end(), order_foreign->begin() + bf[b]);
            for (size_t k = 0; k < X.chunk.size(); k += 2) {
                const int32_t le = X.chunk[k];
                H.tile_chunk[bc[b] + k] = (le & kLeForeign) ? (int32_t)(n_owned + bf[b] + (le & ~kLeForeign)) : (int32_t)(bo[b] + le);
                H.tile_chunk[bc[b] + k + 1] = (int32_t)(bx[b] + X.chunk[k + 1]);
            }
            for (size_t k = 0; k < X.xt.size(); k++) xt[bt[b] + k] = {X.xt[k].first, (int32_t)(bx[b] + X.xt[k].second)};
            for (int64_t t = X.t0; t < X.t1; t++) {
                int32_t *T = &H.tile_tab[8 * (size_t)t];
                T[3] += (int32_t)bm[b];
                T[5] += (int32_t)bh[b];
            }
            X = TileBuf();
        }
    };
    chunked(nb, 1, cp);
    nx = bx[nb];
    return true;
}

}  // namespace

bool build_tiles(const TileInput &in, SpPlanHost &H, std::vector<int32_t> &order, std::vector<int32_t> &order_foreign,
                 std::string &why) {
    const int32_t ng = in.ng;
    const int64_t E = in.E;
    const int32_t *ap = in.ap;
    const int32_t lo = H.lo, hi = H.hi;
    static const int umax = [] {
        const char *e = std::getenv("DEFTRI_SP_TILE_UNITS");
        const int v = e ? std::atoi(e) : kSpTileUnits;
        return std::max(8, std::min(v, 128));
    }();
    static const int64_t lds_budget = [] {
        const char *e = std::getenv("DEFTRI_SP_TILE_LDS");
        return (int64_t)(e ? std::atoi(e) : kSpTileLds);
    }();
    // DEFTRI_PLAN_TIMING: the stages of this build too
    static const bool timing = std::getenv("DEFTRI_PLAN_TIMING") != nullptr;
    auto T0 = std::chrono::steady_clock::now();
    auto lap = [&](const char *w) {
        if (!timing) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[deftri plan]   4a %-26s %8.2f ms\n", w, std::chrono::duration<double, std::milli>(t - T0).count());
        T0 = t;
    };
    // groups: size and first row (rows of a group are consecutive, groups in Morton order); this
    // rank's groups are one range [G0, G1) of that order (ranks are cut at group starts)
    std::vector<int32_t> gsz(ng, 0), grow(ng, INT32_MAX);
    for (int32_t p = 0; p < in.P; p++) {
        const int32_t g = in.gpos[p];
        gsz[g]++;
        grow[g] = std::min(grow[g], in.row_of_point[p]);
    }
    int32_t G0 = ng, G1 = 0;
    for (int32_t g = 0; g < ng; g++) {
        if (gsz[g] > 2) { why = "a keyframe-copy group of more than 2 rows"; return false; }
        if (gsz[g] > 0 && grow[g] >= lo && grow[g] < hi) { G0 = std::min(G0, g); G1 = std::max(G1, g + 1); }
    }
    if (G0 >= G1) { G0 = G1 = 0; }
    for (int32_t g = G0; g < G1; g++)
        if (gsz[g] > 0 && (grow[g] < lo || grow[g] >= hi)) { why = "the rank's groups are not one range"; return false; }
    auto own = [&](int32_t g) { return g >= G0 && g < G1; };
    // the local ARAP edges by group: out-edges of the rank's groups (the owned edges), in-edges of its
    // groups from its groups, and in-edges from other ranks' groups (the halo-only edges: their j
    // vertex is this rank's).  Counting sorts by group over contiguous edge chunks on host threads
    // (per-chunk counts, each chunk's edges after the earlier chunks' — the sequential order)
    std::vector<int32_t> egi(E), egj(E), erow(4 * (size_t)E);
    std::vector<int64_t> ooff(ng + 1, 0), ioff(ng + 1, 0), foff(ng + 1, 0);
    std::vector<int32_t> oe, isrc, fe;
    {
        constexpr int kMaxChunks = 16;
        std::vector<std::vector<int32_t>> co(kMaxChunks), ci(kMaxChunks), cf(kMaxChunks);
        int bad[kMaxChunks] = {0};
        const int nch = chunked(E, 1 << 15, [&](int c, int64_t elo, int64_t ehi) {
            co[c].assign(ng, 0);
            ci[c].assign(ng, 0);
            cf[c].assign(ng, 0);
            for (int64_t e = elo; e < ehi; e++) {
                const int32_t gi = in.gpos[ap[4 * e]], gj = in.gpos[ap[4 * e + 2]];
                egi[e] = gi;
                egj[e] = gj;
                for (int k = 0; k < 4; k++) erow[4 * e + k] = in.row_of_point[ap[4 * e + k]] - lo;
                if (!own(gi) && !own(gj)) continue;
                if (gi != in.gpos[ap[4 * e + 1]] || gj != in.gpos[ap[4 * e + 3]] || gi == gj) bad[c] = 1;
                if (own(gi)) {
                    co[c][gi]++;
                    if (own(gj)) ci[c][gj]++;
                } else {
                    cf[c][gj]++;
                }
            }
        });
        for (int c = 0; c < nch; c++)
            if (bad[c]) { why = "an edge's copies in two groups"; return false; }
        for (int32_t g = 0; g < ng; g++) {
            int64_t so = 0, si = 0, sf = 0;
            for (int c = 0; c < nch; c++) { so += co[c][g]; si += ci[c][g]; sf += cf[c][g]; }
            ooff[g + 1] = ooff[g] + so;
            ioff[g + 1] = ioff[g] + si;
            foff[g + 1] = foff[g] + sf;
        }
        oe.resize(ooff[ng]);
        isrc.resize(ioff[ng]);
        fe.resize(foff[ng]);
        chunked(ng, 1 << 12, [&](int, int64_t glo, int64_t ghi) {
            for (int64_t g = glo; g < ghi; g++) {
                int64_t fo = ooff[g], fi = ioff[g], ff = foff[g];
                for (int c = 0; c < nch; c++) {
                    const int32_t a = co[c][g], b = ci[c][g], f = cf[c][g];
                    co[c][g] = (int32_t)fo;
                    ci[c][g] = (int32_t)fi;
                    cf[c][g] = (int32_t)ff;
                    fo += a;
                    fi += b;
                    ff += f;
                }
            }
        });
        chunked(E, 1 << 15, [&](int c, int64_t elo, int64_t ehi) {
            for (int64_t e = elo; e < ehi; e++) {
                const int32_t gi = egi[e], gj = egj[e];
                if (own(gi)) {
                    oe[co[c][gi]++] = (int32_t)e;
                    if (own(gj)) isrc[ci[c][gj]++] = gi;
                } else if (own(gj)) {
                    fe[cf[c][gj]++] = (int32_t)e;
                }
            }
        });
    }
    // the j group of every out-edge (out-edge order), the i group of every halo-only in-edge
    std::vector<int32_t> okj(oe.size()), fki(fe.size());
    chunked((int64_t)oe.size(), 1 << 15, [&](int, int64_t klo, int64_t khi) {
        for (int64_t k = klo; k < khi; k++) okj[k] = egj[oe[k]];
    });
    for (size_t k = 0; k < fe.size(); k++) fki[k] = egi[fe[k]];
    for (int32_t g = G0; g < G1; g++)
        if (ooff[g + 1] - ooff[g] > 64) { why = "a vertex with more than 64 ARAP edges"; return false; }
    lap("groups, edges by group");
    // (a group with edges holds p1_i and p2_i: 2 rows; a 1-row group has no ARAP edge)
    // 1. greedy partition: consecutive groups while rows <= 2 umax and the LDS estimate fits
    auto lds_of = [&](int64_t nr, int64_t nh, int64_t ns) { return 24 * (nr + nh) + 24 * nr + 24 * ns + kSpTileLdsFixed; };
    std::vector<int32_t> tstart;
    std::vector<int32_t> hcnt(ng, 0), stamp(ng, -1);
    {
        int32_t gs = G0, attempt = 0;
        int64_t nr = 0, nh = 0, ns = 0, units = 0;
        std::vector<int32_t> halo_members;
        tstart.push_back(G0);
        for (int32_t g = G0; g < G1;) {
            // tentative add of g (stamp: the halo groups this attempt already counted)
            int64_t dnh = 0, dns = 0;
            attempt++;
            for (int64_t k = ooff[g]; k < ooff[g + 1]; k++) {
                const int32_t gj = okj[k];
                if (gj >= gs && gj < g) dns += 2;
                else if (hcnt[gj] == 0 && stamp[gj] != attempt) { stamp[gj] = attempt; dnh += gsz[gj]; }
            }
            for (int64_t k = ioff[g]; k < ioff[g + 1]; k++)
                if (isrc[k] >= gs && isrc[k] < g) dns += 2;
            for (int64_t k = foff[g]; k < foff[g + 1]; k++) {       // halo-only in-edges: 2 slots on g
                const int32_t gi = fki[k];
                dns += 2;
                if (hcnt[gi] == 0 && stamp[gi] != attempt) { stamp[gi] = attempt; dnh += gsz[gi]; }
            }
            if (hcnt[g] > 0) dnh -= gsz[g];
            const bool fits = units + 1 <= umax && lds_of(nr + gsz[g], nh + dnh, ns + dns) <= lds_budget &&
                              nr + gsz[g] + nh + dnh < 4096 && ns + dns < 4096;
            if (!fits && units > 0) {
                // close the tile [gs, g): clear its halo counts
                for (int32_t h : halo_members) hcnt[h] = 0;
                halo_members.clear();
                gs = g;
                nr = nh = ns = units = 0;
                tstart.push_back(g);
                continue;
            }
            // commit
            for (int64_t k = ooff[g]; k < ooff[g + 1]; k++) {
                const int32_t gj = okj[k];
                if (!(gj >= gs && gj < g)) {
                    if (hcnt[gj]++ == 0) halo_members.push_back(gj);
                }
            }
            for (int64_t k = foff[g]; k < foff[g + 1]; k++)
                if (hcnt[fki[k]]++ == 0) halo_members.push_back(fki[k]);
            hcnt[g] = 0;                           // g is a tile row now, no longer halo
            nr += gsz[g];
            nh += dnh;
            ns += dns;
            units++;
            g++;
        }
        for (int32_t h : halo_members) hcnt[h] = 0;
        tstart.push_back(G1);
    }
    const int32_t nt = G1 > G0 ? (int32_t)tstart.size() - 1 : 0;
    lap("partition");
    // 2. entries, le order, per tile rows / halo / slots; a tile's owned entries (its vertices'
    //    out-edges) first, then — in chunks of their own — its halo-only entries (other ranks'
    //    vertices' edges into its rows), whose le follow every owned edge's (the plan keeps the owned
    //    edges first)
    H.tile_tab.assign(8 * (size_t)nt, 0);
    order.clear();
    order_foreign.clear();
    const int64_t n_owned = (int64_t)oe.size();
    std::vector<uint32_t> &m0 = H.tile_m0, &m1 = H.tile_m1;
    m0.clear(); m1.clear();
    H.tile_chunk.clear();
    H.tile_halo.clear();
    const int32_t nown = hi - lo;
    H.tile_rs.assign(nown, 0);
    // cross slots: (target row, slot) pairs, CSR by row at the end
    std::vector<std::pair<int32_t, int32_t>> xt;
    int64_t nx = 0;
    int32_t segmax = 1, max_lds = 0;
    std::vector<TileBuf> bufs(16);
    const int nbuf = chunked(nt, 16, [&](int c, int64_t t_lo, int64_t t_hi) {
      TileBuf &B = bufs[c];
      B.t0 = t_lo;
      B.t1 = t_hi;
      std::vector<uint32_t> &m0 = B.m0, &m1 = B.m1;
      std::vector<int32_t> &order = B.order, &order_foreign = B.foreign;
      std::vector<std::pair<int32_t, int32_t>> &xt = B.xt;
      int64_t &nx = B.nx;
      int32_t &segmax = B.segmax, &max_lds = B.max_lds;
      std::vector<int32_t> lrow(ng, -1);          // group -> LDS row base inside the current tile
      std::vector<int32_t> slotcnt, slotfill;     // per tile row
      std::vector<int32_t> hg;
      for (int64_t t = t_lo; t < t_hi; t++) {
        const int32_t g0 = tstart[t], g1 = tstart[t + 1];
        const int32_t r0 = grow[g0] - lo;
        int32_t nr = 0;
        for (int32_t g = g0; g < g1; g++) { lrow[g] = nr; nr += gsz[g]; }
        // halo groups, ascending: out-edges' j groups outside the tile, halo-only edges' i groups
        hg.clear();
        for (int32_t g = g0; g < g1; g++) {
            for (int64_t k = ooff[g]; k < ooff[g + 1]; k++)
                if (okj[k] < g0 || okj[k] >= g1) hg.push_back(okj[k]);
            for (int64_t k = foff[g]; k < foff[g + 1]; k++) hg.push_back(fki[k]);
        }
        std::sort(hg.begin(), hg.end());
        hg.erase(std::unique(hg.begin(), hg.end()), hg.end());
        const int32_t h0 = (int32_t)B.halo.size();
        int32_t nh = 0;
        for (int32_t gj : hg) {
            lrow[gj] = nr + nh;
            for (int32_t k = 0; k < gsz[gj]; k++) B.halo.push_back(grow[gj] + k);   // (global rows)
            nh += gsz[gj];
        }
        // remote slots: count per tile row, in entry order
        slotcnt.assign(nr, 0);
        for (int32_t g = g0; g < g1; g++) {
            for (int64_t k = ooff[g]; k < ooff[g + 1]; k++) {
                const int64_t e = oe[k];
                if (okj[k] >= g0 && okj[k] < g1) {
                    slotcnt[erow[4 * e + 2] - r0]++;
                    slotcnt[erow[4 * e + 3] - r0]++;
                }
            }
            for (int64_t k = foff[g]; k < foff[g + 1]; k++) {
                const int64_t e = fe[k];
                slotcnt[erow[4 * e + 2] - r0]++;
                slotcnt[erow[4 * e + 3] - r0]++;
            }
        }
        slotfill.assign(nr, 0);
        int32_t ns = 0;
        for (int32_t r = 0; r < nr; r++) {
            slotfill[r] = ns;
            if (slotcnt[r] > 0xffff) { B.err = "too many slots on a row"; return; }
            H.tile_rs[r0 + r] = ns | slotcnt[r] << 16;
            ns += slotcnt[r];
        }
        // entries
        const int64_t e0 = (int64_t)m0.size();       // chunk aligned
        int fill = 0;
        auto pad_chunk = [&]() {
            while (fill % 64) {
                m0.push_back(kTmHead);              // padding: its own (empty) segment
                m1.push_back(0);
                fill++;
            }
        };
        auto chunk_start = [&](int64_t le) {
            if (fill % 64 == 0) B.chunk.push_back((int32_t)le), B.chunk.push_back((int32_t)nx);
        };
        for (int32_t g = g0; g < g1; g++) {
            const int64_t k0 = ooff[g], k1 = ooff[g + 1];
            const int cnt = (int)(k1 - k0);
            if (cnt == 0) continue;
            segmax = std::max(segmax, cnt);
            if (fill % 64 + cnt > 64) pad_chunk();
            for (int64_t k = k0; k < k1; k++) {
                chunk_start((int64_t)order.size());
                const int64_t e = oe[k];
                const int32_t gj = okj[k];
                const bool remote = !own(gj);                   // j on another rank: its rows' share there
                const bool cut = !remote && (gj < g0 || gj >= g1);
                const int32_t ra = erow[4 * e] - r0;             // tile rows of p1_i, p2_i
                const int32_t ub = lrow[g];
                const uint32_t swap = ra == ub + 1 ? 1u : 0u;
                // LDS rows of p1_j, p2_j: tile rows, or the halo rows after them
                auto ldsrow = [&](int32_t row) {
                    return (cut || remote) ? lrow[gj] + (row + lo - grow[gj]) : row - r0;
                };
                const uint32_t rj0 = (uint32_t)ldsrow(erow[4 * e + 2]), rj1 = (uint32_t)ldsrow(erow[4 * e + 3]);
                uint32_t w0 = rj0 | rj1 << 12 | kTmValid | swap * kTmSwap;
                if (k == k0) w0 |= kTmHead;
                if (k == k1 - 1) w0 |= kTmLast;
                uint32_t w1 = (uint32_t)ub << 24;
                if (remote) {
                    w0 |= kTmDrop;
                } else if (cut) {
                    w0 |= kTmCut;
                    xt.push_back({erow[4 * e + 2], (int32_t)nx});
                    xt.push_back({erow[4 * e + 3], (int32_t)nx + 1});
                    nx += 2;
                } else {
                    const int32_t s0 = slotfill[rj0]++, s1 = slotfill[rj1]++;
                    w1 |= (uint32_t)s0 | (uint32_t)s1 << 12;
                }
                m0.push_back(w0);
                m1.push_back(w1);
                order.push_back((int32_t)e);
                fill++;
            }
        }
        // halo-only entries, in chunks of their own: each its own segment (no own-row sums); the
        // kernel reads their i rows (halo) through the j fields and their j rows (this tile's)
        // through ub / swap, and writes only the j rows' slots
        bool any_f = false;
        for (int32_t g = g0; g < g1 && !any_f; g++) any_f = foff[g + 1] > foff[g];
        if (any_f) pad_chunk();
        for (int32_t g = g0; g < g1; g++)
            for (int64_t k = foff[g]; k < foff[g + 1]; k++) {
                chunk_start(kLeForeign | (int64_t)order_foreign.size());
                const int64_t e = fe[k];
                const int32_t gi = fki[k];
                const int32_t ub = lrow[g];
                const int32_t rj = erow[4 * e + 2] - r0;        // p1_j's tile row
                const uint32_t swap = rj == ub + 1 ? 1u : 0u;
                const uint32_t ri0 = (uint32_t)(lrow[gi] + (erow[4 * e] + lo - grow[gi]));
                const uint32_t ri1 = (uint32_t)(lrow[gi] + (erow[4 * e + 1] + lo - grow[gi]));
                const uint32_t w0 = ri0 | ri1 << 12 | kTmValid | kTmHead | kTmForeign | swap * kTmSwap;
                const int32_t s0 = slotfill[erow[4 * e + 2] - r0]++, s1 = slotfill[erow[4 * e + 3] - r0]++;
                m0.push_back(w0);
                m1.push_back((uint32_t)s0 | (uint32_t)s1 << 12 | (uint32_t)ub << 24);
                order_foreign.push_back((int32_t)e);
                fill++;
            }
        if (fill == 0) { chunk_start((int64_t)order.size()); m0.push_back(kTmHead); m1.push_back(0); fill = 1; }
        pad_chunk();
        const int64_t ne = (int64_t)m0.size() - e0;
        int32_t *T = &H.tile_tab[8 * (size_t)t];
        T[0] = r0; T[1] = nr; T[2] = nh; T[3] = (int32_t)e0; T[4] = (int32_t)ne; T[5] = h0; T[6] = ns; T[7] = 0;
        max_lds = std::max<int32_t>(max_lds, (int32_t)lds_of(nr, nh, ns));
        for (int32_t g = g0; g < g1; g++) lrow[g] = -1;
        for (int32_t gj : hg) lrow[gj] = -1;
      }
    });
    lap("entries, slots");
    if (!merge_tile_bufs(bufs, nbuf, H, order, &order_foreign, n_owned, xt, nx, segmax, max_lds, why)) return false;
    lap("entries merged");
    if ((int64_t)order.size() != n_owned || order_foreign.size() != fe.size()) { why = "tile order lost edges"; return false; }
    // cross slots by target row, source order inside a row (a counting sort; xt is in source order):
    // the writer scatters its two slots to their destination positions, so a row's slots are one
    // contiguous range the reader sums without an index load
    H.tile_xoff.assign(nown + 1, 0);
    H.tile_xdst.assign(xt.size(), 0);
    for (const auto &x : xt) H.tile_xoff[x.first + 1]++;
    for (int32_t l = 0; l < nown; l++) H.tile_xoff[l + 1] += H.tile_xoff[l];
    {
        std::vector<int32_t> fill(H.tile_xoff.begin(), H.tile_xoff.end() - 1);
        for (const auto &x : xt) H.tile_xdst[x.second] = fill[x.first]++;
    }
    lap("cross slots");
    if (timing) tile_shape_stats(H.tile_tab, nt, nx);
    H.ntile = nt;
    H.tile_entries = (int64_t)m0.size();
    H.tile_cross = nx;
    H.tile_segmax = segmax;
    H.tile_lds = max_lds;
    H.tile_halo_rows = (int64_t)H.tile_halo.size();
    return true;
}

// Several keyframe pairs on one rank (the all-pairs graph of g2oBundleAdjustment.cc:640-645, or its
// window).  A point belongs to the pairs of its keyframe, so a keyframe-copy group holds K rows and
// an ARAP edge of pair q touches the two rows of pair q's keyframes in its i and j groups.  The unit
// is (pair, group): its two rows are the pair's p1_i, p2_i.  Units are ordered by pair, then Morton
// group; tiles are cut per pair exactly as build_tiles cuts one pair's groups (the same LDS budget,
// slots and cross slots), so a tile reads one T_g, one pair's two scales and one W.  A row is an own
// row of one tile per pair containing it: the first of them (its home, share 0) adds the row's
// diagonal terms (D_v + lambda) and stores q; share j > 0 stores its pair's ARAP sums and depth
// couplings in plane j - 1 of a share array, which the update adds to q with the cut edges' slots.
// The plan numbers the rows keyframe-major (spcg_plan.cpp step 3), so a tile's rows are two runs.
bool build_tiles_multi(const TileInput &in, SpPlanHost &H, std::vector<int32_t> &order, std::string &why) {
    const int32_t P = in.P, ng = in.ng, Q = in.Q;
    const int64_t E = in.E;
    const int32_t *ap = in.ap, *row = in.row_of_point;
    static const int umax = [] {
        const char *e = std::getenv("DEFTRI_SP_TILE_UNITS");
        const int v = e ? std::atoi(e) : kSpTileUnits;
        return std::max(8, std::min(v, 128));
    }();
    static const int64_t lds_budget = [] {
        const char *e = std::getenv("DEFTRI_SP_TILE_LDS");
        return (int64_t)(e ? std::atoi(e) : kSpTileLds);
    }();
    static const bool timing = std::getenv("DEFTRI_PLAN_TIMING") != nullptr;
    auto T0 = std::chrono::steady_clock::now();
    auto lap = [&](const char *w) {
        if (!timing) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[deftri plan]   4a %-26s %8.2f ms\n", w, std::chrono::duration<double, std::milli>(t - T0).count());
        T0 = t;
    };
    if (H.nranks != 1) { why = "several pairs on a sharded plan"; return false; }
    if (in.S != 2 * Q) { why = "not two depth scales per pair"; return false; }
    if ((int64_t)Q * ng >= (1LL << 31)) { why = "too many (pair, group) units"; return false; }
    // 1. units (pair, group) with edges, in (pair, Morton group) order; their two rows
    //    (on host threads: a unit's flag and point are the same from every edge of a valid graph; an
    //    invalid one, a unit with two points, fails the row check below whichever edge wrote last)
    std::vector<int32_t> uid((size_t)Q * ng, -1), upt((size_t)Q * ng, -1);
    {
        int bad[16] = {0};
        const int nch = chunked(E, 1 << 16, [&](int c, int64_t e0, int64_t e1) {
            for (int64_t e = e0; e < e1; e++) {
                const int32_t q = in.pair[e];
                if (q < 0 || q >= Q) { bad[c] = 1; return; }
                for (int s = 0; s < 2; s++) {
                    const size_t k = (size_t)q * ng + in.gpos[ap[4 * e + 2 * s]];
                    __atomic_store_n(&uid[k], 0, __ATOMIC_RELAXED);
                    __atomic_store_n(&upt[k], ap[4 * e + 2 * s], __ATOMIC_RELAXED);
                }
            }
        });
        for (int c = 0; c < nch; c++)
            if (bad[c]) { why = "an edge's pair out of range"; return false; }
    }
    int32_t nu = 0;
    if (in.points) {
        // a pair's units in the Morton order of their p1 rows' positions — the pair's own mesh plane
        // (its keyframe 1's positions).  The groups' global Morton order follows one keyframe's
        // positions; cut by it, the other pairs' tiles had twice the halo rows and cut edges (C3: 240
        // halo rows per tile, 36 % of the edges cut, against 124 and 18 % in the pair's own order)
        // pairs on host threads: each pair's units counted, then numbered from the pair's base
        std::vector<int32_t> qb(Q + 1, 0);
        chunked(Q, 1, [&](int, int64_t q0, int64_t q1) {
            for (int64_t q = q0; q < q1; q++)
                for (int32_t g = 0; g < ng; g++) qb[q + 1] += uid[(size_t)q * ng + g] == 0;
        });
        for (int32_t q = 0; q < Q; q++) qb[q + 1] += qb[q];
        nu = qb[Q];
        chunked(Q, 1, [&](int, int64_t q0, int64_t q1) {
          std::vector<std::pair<uint64_t, int32_t>> ks;
          for (int64_t q = q0; q < q1; q++) {
            ks.clear();
            double lo[2] = {1e300, 1e300}, hi[2] = {-1e300, -1e300};
            for (int32_t g = 0; g < ng; g++) {
                const size_t k = (size_t)q * ng + g;
                if (uid[k] != 0) continue;
                for (int c = 0; c < 2; c++) {
                    const double v = in.points[3 * (int64_t)upt[k] + c];
                    lo[c] = std::min(lo[c], v); hi[c] = std::max(hi[c], v);
                }
            }
            for (int32_t g = 0; g < ng; g++) {
                const size_t k = (size_t)q * ng + g;
                if (uid[k] != 0) continue;
                const double *pp = in.points + 3 * (int64_t)upt[k];
                ks.push_back({curve_key(pp[0], pp[1], lo, hi), g});
            }
            std::sort(ks.begin(), ks.end());
            int32_t n = qb[q];
            for (const auto &kg : ks) uid[(size_t)q * ng + kg.second] = n++;
          }
        });
    } else {
        for (size_t k = 0; k < uid.size(); k++)
            if (uid[k] == 0) uid[k] = nu++;
    }
    lap("units");
    std::vector<int32_t> urow(2 * (size_t)nu, -1), upair(nu);
    for (int32_t q = 0; q < Q; q++)
        for (int32_t g = 0; g < ng; g++)
            if (uid[(size_t)q * ng + g] >= 0) upair[uid[(size_t)q * ng + g]] = q;
    // the edges by unit: one pass that sets and checks every unit's rows and counts its out- / in-edges,
    // then a counting sort.  When the edges are pair-major (the graph builder writes them pair by pair)
    // a pair's edges touch only that pair's units, so the pairs run on host threads, each exactly the
    // sequential loop over its own edge range (the first failing pair's first error is the sequential
    // one); otherwise one thread
    std::vector<int32_t> egi(E), egj(E);
    std::vector<int32_t> ocnt(nu + 1, 0), icnt(nu + 1, 0);
    std::vector<int64_t> eb(Q + 1, E);
    bool pair_major = true;
    for (int64_t e = 1; e < E && pair_major; e++) pair_major = in.pair[e] >= in.pair[e - 1];
    if (pair_major) {
        for (int64_t e = E - 1; e >= 0; e--) eb[in.pair[e]] = e;
        for (int32_t q = Q - 1; q >= 0; q--) eb[q] = std::min(eb[q], eb[q + 1]);
    } else {
        std::fill(eb.begin(), eb.end(), E);
        eb[0] = 0;
    }
    const int32_t npart = pair_major ? Q : 1;
    std::vector<const char *> qbad(npart, nullptr);
    chunked(npart, 1, [&](int, int64_t q0, int64_t q1) {
        for (int64_t q = q0; q < q1; q++)
            for (int64_t e = eb[q]; e < eb[q + 1]; e++) {
                const size_t qb = (size_t)in.pair[e] * ng;
                const int32_t ui = uid[qb + in.gpos[ap[4 * e]]], uj = uid[qb + in.gpos[ap[4 * e + 2]]];
                if (ui == uj) { qbad[q] = "an edge inside one group"; break; }
                if (in.gpos[ap[4 * e]] != in.gpos[ap[4 * e + 1]] || in.gpos[ap[4 * e + 2]] != in.gpos[ap[4 * e + 3]]) {
                    qbad[q] = "an edge's copies in two groups";
                    break;
                }
                bool differ = false;
                for (int s = 0; s < 2; s++) {
                    const int32_t u = s ? uj : ui;
                    const int32_t r0 = row[ap[4 * e + 2 * s]], r1 = row[ap[4 * e + 2 * s + 1]];
                    if (urow[2 * (size_t)u] < 0) { urow[2 * (size_t)u] = r0; urow[2 * (size_t)u + 1] = r1; }
                    else if (urow[2 * (size_t)u] != r0 || urow[2 * (size_t)u + 1] != r1) differ = true;
                }
                if (differ) { qbad[q] = "a unit's rows differ between its edges"; break; }
                egi[e] = ui;
                egj[e] = uj;
                ocnt[ui + 1]++;
                icnt[uj + 1]++;
            }
    });
    for (int32_t q = 0; q < npart; q++)
        if (qbad[q]) { why = qbad[q]; return false; }
    for (int32_t u = 0; u < nu; u++) { ocnt[u + 1] += ocnt[u]; icnt[u + 1] += icnt[u]; }
    std::vector<int32_t> oe(E), isrc(E);
    {
        std::vector<int32_t> fo(ocnt.begin(), ocnt.end() - 1), fi(icnt.begin(), icnt.end() - 1);
        chunked(npart, 1, [&](int, int64_t q0, int64_t q1) {
            for (int64_t q = q0; q < q1; q++)
                for (int64_t e = eb[q]; e < eb[q + 1]; e++) {
                    oe[fo[egi[e]]++] = (int32_t)e;
                    isrc[fi[egj[e]]++] = egi[e];
                }
        });
    }
    lap("edges by unit");
    for (int32_t u = 0; u < nu; u++)
        if (ocnt[u + 1] - ocnt[u] > 64) { why = "a vertex with more than 64 ARAP edges in a pair"; return false; }
    // every depth edge's (row, pair of its scale) is a unit's row: it is summed by that unit's tile.
    // A row's unit in pair q is (q, its group); the checks are direct lookups (a sort of every
    // (row, pair) key and a binary search per depth edge took 1.4 s at C3)
    {
        std::vector<int32_t> point_of(P);
        for (int32_t p = 0; p < P; p++) point_of[row[p]] = p;
        // a row in two units of one pair: the unit (q, group of its point) holds it, or it is another
        // group's row — then the row's own (q, group) unit must not list it as well
        for (int32_t u = 0; u < nu; u++)
            for (int k = 0; k < 2; k++) {
                const int32_t r = urow[2 * (size_t)u + k];
                const int32_t uo = uid[(size_t)upair[u] * ng + in.gpos[point_of[r]]];
                if (uo != u) { why = "a row in two units of one pair"; return false; }
            }
        for (int64_t d = 0; d < in.D; d++) {
            const int32_t p = in.dep_point[d], q = in.dep_scale[d] >> 1;
            const int32_t u = (q >= 0 && q < Q) ? uid[(size_t)q * ng + in.gpos[p]] : -1;
            if (u < 0 || (urow[2 * (size_t)u] != row[p] && urow[2 * (size_t)u + 1] != row[p])) {
                why = "a depth edge outside its pair's mesh";
                return false;
            }
        }
        std::vector<uint8_t> seen(P, 0);
        for (int32_t k : urow) seen[k] = 1;
        for (int32_t r = 0; r < P; r++)
            if (!seen[r]) { why = "a row in no pair's mesh"; return false; }
    }
    lap("depth check");
    // 2. greedy partition per pair: consecutive units while units <= umax and the LDS estimate fits
    auto lds_of = [&](int64_t nr, int64_t nh, int64_t ns) { return 24 * (nr + nh) + 24 * nr + 24 * ns + kSpTileLdsFixed; };
    //    A pair's units are one range [pb[q], pb[q + 1]) and its edges stay inside it, so the pairs are
    //    cut independently, on host threads; the tile starts are concatenated in pair order
    std::vector<int32_t> tstart;
    {
        std::vector<int32_t> pb(Q + 1, nu);
        for (int32_t u = nu - 1; u >= 0; u--) pb[upair[u]] = u;
        for (int32_t q = Q - 1; q >= 0; q--) pb[q] = std::min(pb[q], pb[q + 1]);
        int32_t pmax = 0;
        for (int32_t q = 0; q < Q; q++) pmax = std::max(pmax, pb[q + 1] - pb[q]);
        std::vector<std::vector<int32_t>> ts(16);
        const int nts = chunked(Q, 1, [&](int c, int64_t q_lo, int64_t q_hi) {
            std::vector<int32_t> &out = ts[c];
            std::vector<int32_t> hcnt(pmax, 0), stamp(pmax, -1), halo_members;   // by unit - pb[q]
            int32_t attempt = 0;
            for (int64_t q = q_lo; q < q_hi; q++) {
                const int32_t ub = pb[q], ue = pb[q + 1];
                if (ub >= ue) continue;
                int32_t us = ub;
                int64_t nr = 0, nh = 0, ns = 0, units = 0;
                out.push_back(ub);
                for (int32_t u = ub; u < ue;) {
                    int64_t dnh = 0, dns = 0;
                    attempt++;
                    for (int32_t k = ocnt[u]; k < ocnt[u + 1]; k++) {
                        const int32_t uj = egj[oe[k]];
                        if (uj >= us && uj < u) dns += 2;
                        else if (hcnt[uj - ub] == 0 && stamp[uj - ub] != attempt) { stamp[uj - ub] = attempt; dnh += 2; }
                    }
                    for (int32_t k = icnt[u]; k < icnt[u + 1]; k++)
                        if (isrc[k] >= us && isrc[k] < u) dns += 2;
                    if (hcnt[u - ub] > 0) dnh -= 2;
                    const bool fits = units + 1 <= umax && lds_of(nr + 2, nh + dnh, ns + dns) <= lds_budget &&
                                      nr + 2 + nh + dnh < 4096 && ns + dns < 4096;
                    if (!fits && units > 0) {
                        for (int32_t h : halo_members) hcnt[h - ub] = 0;
                        halo_members.clear();
                        us = u;
                        nr = nh = ns = units = 0;
                        out.push_back(u);
                        continue;
                    }
                    for (int32_t k = ocnt[u]; k < ocnt[u + 1]; k++) {
                        const int32_t uj = egj[oe[k]];
                        if (!(uj >= us && uj < u))
                            if (hcnt[uj - ub]++ == 0) halo_members.push_back(uj);
                    }
                    hcnt[u - ub] = 0;
                    nr += 2;
                    nh += dnh;
                    ns += dns;
                    units++;
                    u++;
                }
                for (int32_t h : halo_members) hcnt[h - ub] = 0;
                halo_members.clear();
            }
        });
        for (int c = 0; c < nts; c++) tstart.insert(tstart.end(), ts[c].begin(), ts[c].end());
        if (tstart.empty()) tstart.push_back(0);
        tstart.push_back(nu);
    }
    lap("partition");
    const int32_t nt = nu > 0 ? (int32_t)tstart.size() - 1 : 0;
    // 3. entries, own-row lists, slots, cross slots (the cut edges' first: chunk bases count them)
    H.tile_tab.assign(8 * (size_t)nt, 0);
    H.tile_poff.assign(Q + 1, nt);
    order.clear();
    std::vector<uint32_t> &m0 = H.tile_m0, &m1 = H.tile_m1;
    m0.clear(); m1.clear();
    H.tile_chunk.clear();
    H.tile_halo.clear();
    H.tile_trow.clear();
    H.tile_rs.clear();
    std::vector<std::pair<int32_t, int32_t>> xt;         // (target row, slot id)
    int64_t nx = 0;
    int32_t segmax = 1, max_lds = 0;
    // a tile's rows are units [u0, u1)'s: rows 2 u0 .. 2 u1 of the tile row list (tiles cover the units
    // in order), so each thread writes its tiles' trow / rs ranges in place
    H.tile_trow.assign(2 * (size_t)nu, 0);
    H.tile_rs.assign(2 * (size_t)nu, 0);
    std::vector<TileBuf> bufs(16);
    const int nbuf = chunked(nt, 16, [&](int c, int64_t t_lo, int64_t t_hi) {
      TileBuf &B = bufs[c];
      B.t0 = t_lo;
      B.t1 = t_hi;
      std::vector<uint32_t> &m0 = B.m0, &m1 = B.m1;
      std::vector<int32_t> &order = B.order;
      std::vector<std::pair<int32_t, int32_t>> &xt = B.xt;
      int64_t &nx = B.nx;
      int32_t &segmax = B.segmax, &max_lds = B.max_lds;
      std::vector<int32_t> slotcnt, slotfill, hu;
      for (int64_t t = t_lo; t < t_hi; t++) {
        const int32_t u0 = tstart[t], u1 = tstart[t + 1], q = upair[u0];
        const int32_t nr = 2 * (u1 - u0), r0 = 2 * u0;
        for (int32_t u = u0; u < u1; u++) {
            H.tile_trow[2 * (size_t)u] = urow[2 * (size_t)u];
            H.tile_trow[2 * (size_t)u + 1] = urow[2 * (size_t)u + 1];
        }
        hu.clear();
        for (int32_t u = u0; u < u1; u++)
            for (int32_t k = ocnt[u]; k < ocnt[u + 1]; k++)
                if (egj[oe[k]] < u0 || egj[oe[k]] >= u1) hu.push_back(egj[oe[k]]);
        std::sort(hu.begin(), hu.end());
        hu.erase(std::unique(hu.begin(), hu.end()), hu.end());
        // unit -> LDS row base: the tile's units, then the halo units in ascending order
        auto lrow = [&](int32_t u) {
            return u >= u0 && u < u1 ? 2 * (u - u0) : nr + 2 * (int32_t)(std::lower_bound(hu.begin(), hu.end(), u) - hu.begin());
        };
        const int32_t h0 = (int32_t)B.halo.size();
        const int32_t nh = 2 * (int32_t)hu.size();
        for (size_t k = 0; k < hu.size(); k++) {
            B.halo.push_back(urow[2 * (size_t)hu[k]]);
            B.halo.push_back(urow[2 * (size_t)hu[k] + 1]);
        }
        slotcnt.assign(nr, 0);
        for (int32_t u = u0; u < u1; u++)
            for (int32_t k = ocnt[u]; k < ocnt[u + 1]; k++) {
                const int32_t uj = egj[oe[k]];
                if (uj >= u0 && uj < u1) { slotcnt[2 * (uj - u0)]++; slotcnt[2 * (uj - u0) + 1]++; }
            }
        slotfill.assign(nr, 0);
        int32_t ns = 0;
        for (int32_t r = 0; r < nr; r++) {
            slotfill[r] = ns;
            if (slotcnt[r] > 0xffff) { B.err = "too many slots on a row"; return; }
            H.tile_rs[r0 + r] = ns | slotcnt[r] << 16;
            ns += slotcnt[r];
        }
        const int64_t e0 = (int64_t)m0.size();
        int fill = 0;
        auto pad_chunk = [&]() {
            while (fill % 64) {
                m0.push_back(kTmHead);
                m1.push_back(0);
                fill++;
            }
        };
        for (int32_t u = u0; u < u1; u++) {
            const int32_t k0 = ocnt[u], k1 = ocnt[u + 1];
            const int cnt = k1 - k0;
            if (cnt == 0) continue;
            segmax = std::max(segmax, cnt);
            if (fill % 64 + cnt > 64) pad_chunk();
            for (int32_t k = k0; k < k1; k++) {
                if (fill % 64 == 0) B.chunk.push_back((int32_t)order.size()), B.chunk.push_back((int32_t)nx);
                const int64_t e = oe[k];
                const int32_t uj = egj[e];
                const bool cut = uj < u0 || uj >= u1;
                const uint32_t ub = (uint32_t)(2 * (u - u0));
                const uint32_t rj0 = (uint32_t)lrow(uj), rj1 = rj0 + 1;
                uint32_t w0 = rj0 | rj1 << 12 | kTmValid;
                if (k == k0) w0 |= kTmHead;
                if (k == k1 - 1) w0 |= kTmLast;
                uint32_t w1 = ub << 24;
                if (cut) {
                    w0 |= kTmCut;
                    xt.push_back({row[ap[4 * e + 2]], (int32_t)nx});
                    xt.push_back({row[ap[4 * e + 3]], (int32_t)nx + 1});
                    nx += 2;
                } else {
                    const int32_t s0 = slotfill[rj0]++, s1 = slotfill[rj1]++;
                    w1 |= (uint32_t)s0 | (uint32_t)s1 << 12;
                }
                m0.push_back(w0);
                m1.push_back(w1);
                order.push_back((int32_t)e);
                fill++;
            }
        }
        if (fill == 0) { B.chunk.push_back((int32_t)order.size()); B.chunk.push_back((int32_t)nx); m0.push_back(kTmHead); m1.push_back(0); fill = 1; }
        pad_chunk();
        const int64_t ne = (int64_t)m0.size() - e0;
        if (nr > 256) { B.err = "a tile of more than 128 units"; return; }   // (ub: 8 bits)
        int32_t *T = &H.tile_tab[8 * (size_t)t];
        T[0] = r0; T[1] = nr; T[2] = nh; T[3] = (int32_t)e0; T[4] = (int32_t)ne; T[5] = h0; T[6] = ns; T[7] = q;
        max_lds = std::max<int32_t>(max_lds, (int32_t)lds_of(nr, nh, ns));
      }
    });
    lap("entries, slots");
    if (!merge_tile_bufs(bufs, nbuf, H, order, nullptr, 0, xt, nx, segmax, max_lds, why)) return false;
    for (int32_t t = 0; t < nt; t++)
        if (H.tile_poff[H.tile_tab[8 * (size_t)t + 7]] == nt) H.tile_poff[H.tile_tab[8 * (size_t)t + 7]] = t;
    lap("entries merged");
    for (int32_t q = Q - 1; q >= 0; q--)
        if (H.tile_poff[q] == nt) H.tile_poff[q] = H.tile_poff[q + 1];
    if ((int64_t)order.size() != E) { why = "tile order lost edges"; return false; }
    // 4. shares: a row's tiles in tile (= pair) order are its shares 0, 1, ...; share 0 (the home)
    //    adds the row's diagonal terms and stores q, share j > 0 its pair's sums in plane j - 1 of the
    //    share array (row-major per plane, so a tile's stores and the update's loads coalesce)
    H.tile_tdst.assign(H.tile_trow.size(), 0);
    H.tile_nshare.assign(P, 0);
    for (size_t k = 0; k < H.tile_trow.size(); k++) {
        const int32_t r = H.tile_trow[k];
        const int32_t j = H.tile_nshare[r]++;
        H.tile_tdst[k] = j;
        if (j == 0) H.tile_trow[k] = r | (int32_t)(1u << 31);
    }
    lap("shares");
    H.tile_planes = 0;
    for (int32_t c : H.tile_nshare) H.tile_planes = std::max(H.tile_planes, c - 1);
    // cross slots by target row, source order inside a row
    H.tile_xoff.assign(P + 1, 0);
    H.tile_xdst.assign(xt.size(), 0);
    for (const auto &x : xt) H.tile_xoff[x.first + 1]++;
    for (int32_t l = 0; l < P; l++) H.tile_xoff[l + 1] += H.tile_xoff[l];
    {
        std::vector<int32_t> fill(H.tile_xoff.begin(), H.tile_xoff.end() - 1);
        for (const auto &x : xt) H.tile_xdst[x.second] = fill[x.first]++;
    }
    lap("cross slots");
    if (timing) tile_shape_stats(H.tile_tab, nt, nx);
    H.tile_multi = true;
    H.ntile = nt;
    H.tile_entries = (int64_t)m0.size();
    H.tile_cross = nx;
    H.tile_segmax = segmax;
    H.tile_lds = max_lds;
    H.tile_halo_rows = (int64_t)H.tile_halo.size();
    return true;
}

}  // namespace deftri

namespace deftri {

// Host emulation of one tile-mode product q = (H + lambda I) p (tests, no GPU): k_sp_tile's entry
// walk — le and cross slots from the chunk bases and the valid / cut lanes before an entry, the own
// rows' sums, the LDS remote slots and the cross slots — then the update's cross sums, with the
// layout checked on the way: every LDS slot and every cross slot written exactly once and read exactly
// once, every local edge visited once (owned ones in the owned range, halo-only ones after it).
// J / W in the problem's edge order; q in problem order: this rank's rows, and the heavy rows' sums
// over its owned edges and own depth edges (+ lambda p on one rank; a sharded caller all-reduces them
// and adds it).  Returns 0, or -1 (why) on a layout fault.
int sp_emulate_tile_product(const deftri_problem_desc &d, const SpPlanHost &H, const double *Ja, const double *Wa,
                            const double *Jr, const double *Wr, const double *Jd, const double *Wd, double lambda,
                            const double *p, double *q, std::string &why) {
    if (!H.tile) { why = "not a tile plan"; return -1; }
    const int64_t hd = H.hd, ndof = hd + 3 * (int64_t)H.P;
    const int32_t Q = H.Q, nown = H.hi - H.lo, lo = H.lo;
    std::vector<double> pl(ndof, 0.0), qr(ndof, 0.0);
    for (int64_t k = 0; k < hd; k++) pl[k] = p[k];
    for (int32_t r = 0; r < H.P; r++)
        for (int c = 0; c < 3; c++) pl[hd + 3 * (int64_t)r + c] = p[hd + 3 * (int64_t)H.point_of_row[r] + c];
    std::vector<double> hsum(hd, 0.0), xc(3 * std::max<int64_t>(H.tile_cross, 1), 0.0);
    std::vector<int> xw(std::max<int64_t>(H.tile_cross, 1), 0), xr(std::max<int64_t>(H.tile_cross, 1), 0);
    std::vector<int> lew(H.arap_ids.size(), 0);
    std::vector<int> dw(d.n_depth, 0);                   // every depth edge summed exactly once
    const bool multi = H.tile_multi;
    std::vector<double> qs(3 * (size_t)std::max(H.tile_planes, 0) * nown, 0.0);   // share planes
    std::vector<int> sw_((size_t)std::max(H.tile_planes, 0) * nown, 0);
    for (int32_t t = 0; t < H.ntile; t++) {
        const int32_t *T = &H.tile_tab[8 * (size_t)t];
        const int32_t r0 = T[0], nr = T[1], nh = T[2], e0 = T[3], ne = T[4], h0 = T[5], ns = T[6], tq = T[7];
        if (e0 % 64 || ne % 64) { why = "tile entries not chunk aligned"; return -1; }
        if (multi && (t < H.tile_poff[tq] || t >= H.tile_poff[tq + 1])) { why = "a tile outside its pair's range"; return -1; }
        std::vector<double> pL(3 * (size_t)(nr + nh)), up(3 * (size_t)nr, 0.0), rs(3 * (size_t)std::max(ns, 1), 0.0);
        std::vector<int> rsw(std::max(ns, 1), 0), rsr(std::max(ns, 1), 0);
        auto grow_of = [&](int32_t i) {
            return i < nr ? (multi ? (H.tile_trow[r0 + i] & 0x7fffffff) : lo + r0 + i) : H.tile_halo[h0 + i - nr];
        };
        for (int32_t i = 0; i < nr + nh; i++)
            for (int c = 0; c < 3; c++) pL[3 * (size_t)i + c] = pl[hd + 3 * (int64_t)grow_of(i) + c];
        int nv = 0, nc = 0;
        for (int32_t k = 0; k < ne; k++) {
            const int64_t ke = (int64_t)e0 + k;
            if ((ke & 63) == 0) nv = nc = 0;
            const uint32_t m0 = H.tile_m0[ke], m1 = H.tile_m1[ke];
            const int32_t *ch = &H.tile_chunk[2 * (size_t)(ke >> 6)];
            if (!(m0 & kTmValid)) continue;
            const int64_t le = ch[0] + nv++;
            const bool cut = (m0 & kTmCut) != 0, foreign = (m0 & kTmForeign) != 0, drop = (m0 & kTmDrop) != 0;
            const int64_t x = ch[1] + 2 * (int64_t)(cut ? nc++ : nc);
            if (le >= (int64_t)H.arap_ids.size()) { why = "le out of range"; return -1; }
            if (foreign != (le >= H.n_arap_owned)) { why = "an entry's le outside its class's range"; return -1; }
            lew[le]++;
            const int64_t e = H.arap_ids[le];
            const double *J = Ja + 18 * e;
            if (multi && d.arap_pair[e] != tq) { why = "an entry of another pair"; return -1; }
            const int ub = (int)(m1 >> 24), sw = (int)((m0 >> 26) & 1u);
            const int ro0 = ub + sw, ro1 = ub + 1 - sw, rf0 = (int)(m0 & 0xfffu), rf1 = (int)((m0 >> 12) & 0xfffu);
            const int rows[4] = {foreign ? rf0 : ro0, foreign ? rf1 : ro1, foreign ? ro0 : rf0, foreign ? ro1 : rf1};
            for (int kk = 0; kk < 4; kk++) {
                const bool tile_row = foreign ? kk >= 2 : kk < 2;
                const int32_t lim = tile_row ? nr : nr + nh;
                if (rows[kk] < 0 || rows[kk] >= lim) { why = "an entry's LDS row out of range"; return -1; }
                // the LDS row must hold the edge's point
                if (H.row_of_point[d.arap_pts[4 * e + kk]] != grow_of(rows[kk])) { why = "an entry's LDS row is not its point's row"; return -1; }
            }
            double tt = 0.0;
            for (int kk = 0; kk < 4; kk++)
                for (int c = 0; c < 3; c++) tt += J[3 * kk + c] * pL[3 * (size_t)rows[kk] + c];
            for (int c = 0; c < 6; c++) tt += J[12 + c] * pl[6 * (int64_t)d.arap_pair[e] + c];
            const double s = Wa[e] * tt;
            if (!foreign) {
                for (int c = 0; c < 6; c++) hsum[6 * (int64_t)d.arap_pair[e] + c] += J[12 + c] * s;
                for (int c = 0; c < 3; c++) { up[3 * (size_t)rows[0] + c] += J[c] * s; up[3 * (size_t)rows[1] + c] += J[3 + c] * s; }
            }
            if (drop) continue;
            if (cut) {
                if (x < 0 || x + 2 > H.tile_cross) { why = "cross slot out of range"; return -1; }
                const int64_t d0 = H.tile_xdst[x], d1 = H.tile_xdst[x + 1];
                xw[d0]++; xw[d1]++;
                for (int c = 0; c < 3; c++) { xc[3 * d0 + c] = J[6 + c] * s; xc[3 * d1 + c] = J[9 + c] * s; }
            } else {
                const int s0 = (int)(m1 & 0xfffu), s1 = (int)((m1 >> 12) & 0xfffu);
                if (s0 >= ns || s1 >= ns) { why = "LDS slot out of range"; return -1; }
                rsw[s0]++; rsw[s1]++;
                for (int c = 0; c < 3; c++) { rs[3 * (size_t)s0 + c] = J[6 + c] * s; rs[3 * (size_t)s1 + c] = J[9 + c] * s; }
            }
        }
        for (int32_t tr = 0; tr < nr; tr++) {
            const int32_t l = multi ? (H.tile_trow[r0 + tr] & 0x7fffffff) - lo : r0 + tr;
            const bool home = !multi || H.tile_trow[r0 + tr] < 0;
            const int rsi = H.tile_rs[r0 + tr], sb = rsi & 0xffff, sc = rsi >> 16;
            double acc[3];
            for (int c = 0; c < 3; c++) acc[c] = up[3 * (size_t)tr + c] + (home ? lambda * pL[3 * (size_t)tr + c] : 0.0);
            for (int k = sb; k < sb + sc; k++) {
                if (k >= ns) { why = "row slot range out of range"; return -1; }
                rsr[k]++;
                for (int c = 0; c < 3; c++) acc[c] += rs[3 * (size_t)k + c];
            }
            const int64_t o = hd + 3 * (int64_t)(lo + l);
            for (int32_t j = home ? H.rep_off[l] : 0; home && j < H.rep_off[l + 1]; j++) {
                const int64_t e = H.rep_ids[j];
                const double *J = Jr + 6 * e;
                for (int rr = 0; rr < 2; rr++) {
                    double tt = 0;
                    for (int c = 0; c < 3; c++) tt += J[3 * rr + c] * pl[o + c];
                    for (int c = 0; c < 3; c++) acc[c] += J[3 * rr + c] * Wr[e] * tt;
                }
            }
            for (int32_t j = H.dep_off[l]; j < H.dep_off[l + 1]; j++) {
                const int64_t e = H.dep_ids[j];
                const double *J = Jd + 4 * e;
                const int32_t sc_ = d.dep_scale[e];
                if (multi && (sc_ >> 1) != tq) continue;  // another pair's tile sums it
                dw[e]++;
                double tt = J[3] * pl[6 * (int64_t)Q + sc_];
                for (int c = 0; c < 3; c++) tt += J[c] * pl[o + c];
                for (int c = 0; c < 3; c++) acc[c] += J[c] * Wd[e] * tt;
                hsum[6 * (int64_t)Q + sc_] += J[3] * Wd[e] * tt;
            }
            if (home) {
                for (int c = 0; c < 3; c++) qr[o + c] = acc[c];
            } else {
                const int64_t j = H.tile_tdst[r0 + tr];
                if (j < 1 || j > H.tile_planes) { why = "a share's plane out of range"; return -1; }
                const int64_t x = (j - 1) * nown + l;
                if (sw_[x]++) { why = "a share written twice"; return -1; }
                for (int c = 0; c < 3; c++) qs[3 * x + c] = acc[c];
            }
        }
        for (int32_t k = 0; k < ns; k++)
            if (rsw[k] != 1 || rsr[k] != 1) { why = "an LDS slot not written / read exactly once"; return -1; }
    }
    for (size_t le = 0; le < lew.size(); le++)
        if (lew[le] != 1) { why = "a local edge not visited exactly once"; return -1; }
    if (H.nranks <= 1)
        for (int64_t e = 0; e < d.n_depth; e++)
            if (dw[e] != 1) { why = "a depth edge not summed exactly once"; return -1; }
    for (int32_t l = 0; l < nown && multi; l++)                 // the update: q + the row's shares
        for (int32_t j = 1; j < H.tile_nshare[lo + l]; j++) {
            const int64_t x = (int64_t)(j - 1) * nown + l;
            if (sw_[x] != 1) { why = "a share not written exactly once"; return -1; }
            for (int c = 0; c < 3; c++) qr[hd + 3 * (int64_t)(lo + l) + c] += qs[3 * x + c];
        }
    for (int32_t l = 0; l < nown; l++)
        for (int32_t k = H.tile_xoff[l]; k < H.tile_xoff[l + 1]; k++) {
            const int64_t x = k;
            xr[x]++;
            for (int c = 0; c < 3; c++) qr[hd + 3 * (int64_t)(lo + l) + c] += xc[3 * x + c];
        }
    for (int64_t x = 0; x < H.tile_cross; x++)
        if (xw[x] != 1 || xr[x] != 1) { why = "a cross slot not written / read exactly once"; return -1; }
    for (int64_t k = 0; k < ndof; k++) q[k] = 0.0;
    for (int32_t l = 0; l < nown; l++)
        for (int c = 0; c < 3; c++) q[hd + 3 * (int64_t)H.point_of_row[lo + l] + c] = qr[hd + 3 * (int64_t)(lo + l) + c];
    const bool one = H.nranks <= 1;
    for (int64_t k = 0; k < hd; k++) q[k] = hsum[k] + (one ? lambda * pl[k] : 0.0);
    return 0;
}

}  // namespace deftri
