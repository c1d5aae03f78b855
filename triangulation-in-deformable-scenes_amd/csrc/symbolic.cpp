// symbolic.cpp — nested-dissection ordering + multifrontal plan (see symbolic.h).
#include "symbolic.h"

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <numeric>
#include <thread>
#include <unordered_set>

namespace deftri {

namespace {

struct Builder {
    const deftri_problem_desc &d;
    Symbolic &S;
    int leaf;
    int32_t Q, NS, P;
    std::vector<int64_t> adj_begin;       // vertex adjacency CSR (sorted, unique, no self)
    std::vector<int64_t> adj;
    std::vector<double> xy;               // point ordering coordinates
    // front construction
    std::vector<std::vector<int64_t>> own;        // per front: own vertices (elim order)
    std::vector<std::vector<int64_t>> bnd;        // per front: boundary vertices (elim order)
    std::vector<int32_t> vfront;                  // vertex -> owning front
    int64_t next_pos = 0;
    // per-thread scratch of the nested dissection, indexed by point (the subdomains of concurrent
    // tasks are disjoint, but their separator searches read the neighbours' sides)
    struct Scratch {
        std::vector<int32_t> side;
        std::vector<int32_t> stamp;      // distinct-count scratch
        int32_t stamp_id = 0;
        std::vector<int64_t> spos;       // index of a point in the separator list being refined
        explicit Scratch(int32_t n) : side(std::max(n, 1), 0), stamp(std::max(n, 1), 0), spos(std::max(n, 1), -1) {}
    };
    // dissection tree under construction: fronts in postorder (own vertices, children; -1 = none)
    struct LocalTree {
        std::vector<std::vector<int64_t>> own;
        std::vector<std::array<int32_t, 2>> ch;
        int32_t add(std::vector<int64_t> &&ov, int32_t c0, int32_t c1) {
            own.push_back(std::move(ov));
            ch.push_back({c0, c1});
            return (int32_t)own.size() - 1;
        }
        int32_t append(LocalTree &&o) {          // o's fronts after ours; returns the index offset
            const int32_t off = (int32_t)own.size();
            for (size_t i = 0; i < o.own.size(); i++) {
                own.push_back(std::move(o.own[i]));
                ch.push_back({o.ch[i][0] < 0 ? -1 : o.ch[i][0] + off, o.ch[i][1] < 0 ? -1 : o.ch[i][1] + off});
            }
            return off;
        }
    };
    int nd_dirs = 4;
    int nd_passes = 8;
    int nd_try = 3;
    double nd_bal = 0.55;

    int rank = 0, nranks = 1;
    int par_depth = 3;                   // dissection levels whose halves run concurrently (2^3 threads)
    static constexpr int64_t par_min = 4096;   // smallest subdomain worth a thread
    Builder(const deftri_problem_desc &d_, Symbolic &S_, int leaf_, int rank_, int nranks_)
        : d(d_), S(S_), leaf(leaf_), rank(rank_), nranks(nranks_) {
        Q = d.n_pairs; NS = d.n_scales; P = d.n_points;
    }

    int64_t vT(int q) const { return q; }
    int64_t vS(int k) const { return (int64_t)Q + k; }
    int64_t vP(int p) const { return (int64_t)Q + NS + p; }

    // vertex adjacency (sorted, unique, no self): bucket the coupled pairs by vertex, then sort and
    // deduplicate every vertex's list (threads over vertex ranges)
    void build_adjacency() {
        const int64_t nv = S.nv;
        auto each_pair = [&](auto &&fn) {
            for (int e = 0; e < d.n_depth; e++) {
                int64_t a = vP(d.dep_point[e]), b = vS(d.dep_scale[e]);
                fn(a, b); fn(b, a);
            }
            for (int e = 0; e < d.n_arap; e++) {
                int64_t v[5];
                for (int k = 0; k < 4; k++) v[k] = vP(d.arap_pts[4 * (int64_t)e + k]);
                v[4] = vT(d.arap_pair[e]);
                for (int i = 0; i < 5; i++)
                    for (int j = 0; j < 5; j++)
                        if (i != j && v[i] != v[j]) fn(v[i], v[j]);
            }
        };
        std::vector<int64_t> cnt(nv + 1, 0);
        each_pair([&](int64_t a, int64_t) { cnt[a + 1]++; });
        for (int64_t v = 0; v < nv; v++) cnt[v + 1] += cnt[v];
        std::vector<int64_t> raw((size_t)cnt[nv]);
        {
            std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
            each_pair([&](int64_t a, int64_t b) { raw[pos[a]++] = b; });
        }
        std::vector<int64_t> len(nv, 0);
        const int nt = (int)std::max<unsigned>(1, std::min<unsigned>(8, std::thread::hardware_concurrency()));
        auto work = [&](int t) {
            for (int64_t v = t; v < nv; v += nt) {
                auto b = raw.begin() + cnt[v], e = raw.begin() + cnt[v + 1];
                std::sort(b, e);
                len[v] = std::unique(b, e) - b;
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < nt; t++) th.emplace_back(work, t);
        work(0);
        for (auto &x : th) x.join();
        adj_begin.assign(nv + 1, 0);
        for (int64_t v = 0; v < nv; v++) adj_begin[v + 1] = adj_begin[v] + len[v];
        adj.resize((size_t)adj_begin[nv]);
        for (int64_t v = 0; v < nv; v++)
            std::copy(raw.begin() + cnt[v], raw.begin() + cnt[v] + len[v], adj.begin() + adj_begin[v]);
    }

    int32_t new_front(std::vector<int64_t> &&ownv, std::vector<int32_t> children) {
        int32_t f = (int32_t)S.fronts.size();
        Front F{};
        F.parent = -1;
        F.nchild = (int32_t)children.size();
        F.child[0] = F.child[1] = -1;
        for (size_t i = 0; i < children.size(); i++) { F.child[i] = children[i]; S.fronts[children[i]].parent = f; }
        S.fronts.push_back(F);
        for (int64_t v : ownv) { S.elim_pos[v] = next_pos++; vfront[v] = f; }
        own.push_back(std::move(ownv));
        bnd.emplace_back();
        return f;
    }

    // Fiduccia-Mattheyses-style vertex-separator refinement on the current subdomain (side[] = 1/2 for
    // the halves, 3 for the separator).  A move takes a separator point to one half and pulls its
    // neighbours in the other half into the separator (size change: -1 + that count).  Each pass
    // makes the best balanced move repeatedly (hill-climbing through non-positive gains, moved
    // points locked) and rolls back to the smallest separator seen.
    void refine_sep(std::vector<int64_t> &sep, int64_t &nA, int64_t &nB, int64_t ntot, Scratch &sc) {
        auto &side = sc.side; auto &stamp = sc.stamp; auto &spos = sc.spos;
        const int64_t cap = (int64_t)std::ceil(nd_bal * (double)ntot);
        for (size_t i = 0; i < sep.size(); i++) spos[sep[i]] = (int64_t)i;
        auto sep_add = [&](int64_t u) { spos[u] = (int64_t)sep.size(); sep.push_back(u); };
        auto sep_del = [&](int64_t u) {
            int64_t i = spos[u], last = sep.back();
            sep[i] = last; spos[last] = i; sep.pop_back(); spos[u] = -1;
        };
        auto nbrs = [&](int64_t v, auto &&fn) {
            int64_t gv = vP((int32_t)v);
            for (int64_t k = adj_begin[gv]; k < adj_begin[gv + 1]; k++) {
                int64_t u = adj[k] - ((int64_t)Q + NS);
                if (u >= 0) fn(u);
            }
        };
        struct Move { int64_t v; int t; size_t p0, p1; };
        for (int pass = 0; pass < nd_passes; pass++) {
            std::vector<Move> log;
            std::vector<int64_t> pulled;
            size_t best_len = 0;
            int64_t best_sz = (int64_t)sep.size(), best_imb = std::llabs(nA - nB);
            const int32_t lock = ++sc.stamp_id;
            const int64_t maxsteps = (int64_t)sep.size();
            for (int64_t step = 0; step < maxsteps; step++) {
                int64_t bv = -1, bg = 0, bimb = 0;
                int bt = 0;
                for (int64_t v : sep) {
                    if (stamp[v] == lock) continue;
                    int64_t cA = 0, cB = 0;
                    nbrs(v, [&](int64_t u) { cA += side[u] == 1; cB += side[u] == 2; });
                    for (int t = 1; t <= 2; t++) {
                        const int64_t k = t == 1 ? cB : cA;
                        const int64_t a2 = t == 1 ? nA + 1 : nA - cA, b2 = t == 1 ? nB - cB : nB + 1;
                        if (std::max(a2, b2) > cap || std::min(a2, b2) < 1) continue;
                        const int64_t g = 1 - k, imb = std::llabs(a2 - b2);
                        if (bv < 0 || g > bg || (g == bg && imb < bimb)) { bv = v; bt = t; bg = g; bimb = imb; }
                    }
                }
                if (bv < 0) break;
                const int other = 3 - bt;
                sep_del(bv);
                side[bv] = bt;
                stamp[bv] = lock;
                const size_t p0 = pulled.size();
                nbrs(bv, [&](int64_t u) { if (side[u] == other) { side[u] = 3; sep_add(u); pulled.push_back(u); } });
                const int64_t k = (int64_t)(pulled.size() - p0);
                if (bt == 1) { nA += 1; nB -= k; } else { nB += 1; nA -= k; }
                log.push_back({bv, bt, p0, pulled.size()});
                const int64_t sz = (int64_t)sep.size(), imb = std::llabs(nA - nB);
                if (sz < best_sz || (sz == best_sz && imb < best_imb)) { best_sz = sz; best_imb = imb; best_len = log.size(); }
            }
            for (size_t i = log.size(); i > best_len; i--) {      // roll back past the best state
                const Move &m = log[i - 1];
                const int other = 3 - m.t;
                for (size_t j = m.p0; j < m.p1; j++) { side[pulled[j]] = other; sep_del(pulled[j]); }
                const int64_t k = (int64_t)(m.p1 - m.p0);
                if (m.t == 1) { nA -= 1; nB += k; } else { nB -= 1; nA += k; }
                side[m.v] = 3;
                sep_add(m.v);
            }
            if (best_len == 0) break;
        }
        for (int64_t p : sep) spos[p] = -1;
    }

    // nested dissection of `nodes` into T (postorder); returns the subtree's root.  The two halves of
    // a large subdomain near the top are dissected concurrently (left on a new thread with its own
    // scratch, right here) and appended in the sequential order, so the tree — and every elimination
    // position — is the same as a one-thread run.
    int32_t nd(std::vector<int64_t> &nodes, int depth, Scratch &sc, LocalTree &T) {
        auto &side = sc.side;
        int64_t n = (int64_t)nodes.size();
        if (n <= leaf || depth > 48) {
            std::vector<int64_t> o(nodes.begin(), nodes.end());
            std::sort(o.begin(), o.end());
            std::vector<int64_t> ov;
            for (int64_t p : o) ov.push_back(vP((int32_t)p));
            return T.add(std::move(ov), -1, -1);
        }
        // vertex separator: order along a direction, cut, take the boundary vertices of one side (the
        // cut edges need one endpoint each).  Four directions (x, y, both diagonals) x three cut
        // positions (45/50/55 %) x two sides are candidates; the nd_try smallest are refined
        // (refine_sep) and the smallest refined separator wins.
        auto boundary = [&](int64_t cut, bool left, std::vector<int64_t> *out) -> int64_t {
            for (int64_t i = 0; i < n; i++) side[nodes[i]] = (i < cut) ? 1 : 2;
            const int other = left ? 2 : 1;
            int64_t cnt = 0;
            for (int64_t i = left ? 0 : cut; i < (left ? cut : n); i++) {
                int64_t v = vP((int32_t)nodes[i]);
                for (int64_t k = adj_begin[v]; k < adj_begin[v + 1]; k++) {
                    int64_t u = adj[k] - ((int64_t)Q + NS);
                    if (u >= 0 && side[u] == other) { cnt++; if (out) out->push_back(nodes[i]); break; }
                }
            }
            return cnt;
        };
        const int ND_DIRS = nd_dirs;
        double dirs[16][2];
        for (int d = 0; d < ND_DIRS; d++) { dirs[d][0] = std::cos(M_PI * d / ND_DIRS); dirs[d][1] = std::sin(M_PI * d / ND_DIRS); }
        // membership of the k smallest (key, index) is all a cut needs: nth_element, O(n) per cut
        auto place = [&](int d, int64_t lo, int64_t hi, int64_t cut) {
            auto less = [&](int64_t a, int64_t b) {
                double x = dirs[d][0] * xy[2 * a] + dirs[d][1] * xy[2 * a + 1];
                double y = dirs[d][0] * xy[2 * b] + dirs[d][1] * xy[2 * b + 1];
                return x < y || (x == y && a < b);
            };
            std::nth_element(nodes.begin() + lo, nodes.begin() + cut, nodes.begin() + hi, less);
        };
        struct Cand { double score; int d; int64_t cut; bool left; };
        std::vector<Cand> cands;
        const int64_t c50 = n / 2, c45 = (n * 9) / 20, c55 = (n * 11) / 20;
        for (int d = 0; d < ND_DIRS; d++) {
            place(d, 0, n, c50);
            if (c45 > 0) place(d, 0, c50, c45);
            if (c55 < n && c55 > c50) place(d, c50, n, c55);
            for (int64_t cut : {c50, c45, c55}) {
                if (cut <= 0 || cut >= n) continue;
                for (bool left : {true, false}) {
                    const double score = (double)boundary(cut, left, nullptr);
                    cands.push_back({score, d, cut, left});
                }
            }
        }
        std::stable_sort(cands.begin(), cands.end(), [](const Cand &a, const Cand &b) { return a.score < b.score; });
        // the separator of candidate c, refined; side[] left set for the subdomain
        std::vector<int64_t> sep;
        auto realise = [&](const Cand &c) {
            place(c.d, 0, n, c.cut);
            sep.clear();
            boundary(c.cut, c.left, &sep);
            for (int64_t i = 0; i < n; i++) side[nodes[i]] = (i < c.cut) ? 1 : 2;
            for (int64_t p : sep) side[p] = 3;
            if (nd_passes > 0) {
                int64_t nA = 0, nB = 0;
                for (int64_t p : nodes) { nA += side[p] == 1; nB += side[p] == 2; }
                refine_sep(sep, nA, nB, n, sc);
            }
        };
        size_t best = 0;
        const size_t ntry = std::min(cands.size(), (size_t)std::max(1, nd_try));
        if (ntry > 1) {
            size_t best_sz = SIZE_MAX;
            for (size_t c = 0; c < ntry; c++) {
                realise(cands[c]);
                if (sep.size() < best_sz) { best_sz = sep.size(); best = c; }
                for (int64_t p : nodes) side[p] = 0;
            }
        }
        realise(cands[best]);
        const int ax = cands[best].d;
        std::vector<int64_t> L, R, Sp;
        for (int64_t p : nodes) {
            if (side[p] == 1) L.push_back(p);
            else if (side[p] == 2) R.push_back(p);
            else Sp.push_back(p);
        }
        for (int64_t p : nodes) side[p] = 0;
        if (std::getenv("DEFTRI_DEBUG_PLAN") && depth < 3) std::fprintf(stderr, "[nd] depth %d n %lld L %zu R %zu S %zu ax %d\n", depth, (long long)n, L.size(), R.size(), Sp.size(), ax);
        if (L.empty() || R.empty()) {          // cannot split (degenerate coordinates)
            std::vector<int64_t> ov;
            std::sort(nodes.begin(), nodes.end());
            for (int64_t p : nodes) ov.push_back(vP((int32_t)p));
            return T.add(std::move(ov), -1, -1);
        }
        int32_t cl, cr;
        if (depth < par_depth && n >= par_min) {
            LocalTree TL, TR;
            int32_t rl = -1;
            std::thread th([&] { Scratch sl(P); rl = nd(L, depth + 1, sl, TL); });
            const int32_t rr = nd(R, depth + 1, sc, TR);
            th.join();
            cl = T.append(std::move(TL)) + rl;
            cr = T.append(std::move(TR)) + rr;
        } else {
            cl = nd(L, depth + 1, sc, T);
            cr = nd(R, depth + 1, sc, T);
        }
        std::sort(Sp.begin(), Sp.end());
        std::vector<int64_t> ov;
        for (int64_t p : Sp) ov.push_back(vP((int32_t)p));
        return T.add(std::move(ov), cl, cr);
    }

    // phase timing of the analysis (DEFTRI_DEBUG_TIME)
    std::chrono::steady_clock::time_point t_last = std::chrono::steady_clock::now();
    bool dbg_time = std::getenv("DEFTRI_DEBUG_TIME") != nullptr;
    void tick(const char *what) {
        if (!dbg_time) return;
        auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[analyse] %-24s %8.3f s\n", what, std::chrono::duration<double>(now - t_last).count());
        t_last = now;
    }

    bool run() {
        S.nv = (int64_t)Q + NS + P;
        S.vdim.resize(S.nv);
        S.voff.resize(S.nv);
        int64_t off = 0;
        for (int64_t v = 0; v < S.nv; v++) {
            int dim = v < Q ? 6 : (v < Q + NS ? 1 : 3);
            S.vdim[v] = dim; S.voff[v] = off; off += dim;
        }
        S.ndof = off;
        S.elim_pos.assign(S.nv, -1);
        vfront.assign(S.nv, -1);
        build_adjacency();
        tick("adjacency");
        xy.resize(2 * (size_t)std::max(P, 1));
        for (int32_t p = 0; p < P; p++) {
            if (d.order_xy) { xy[2 * p] = d.order_xy[2 * p]; xy[2 * p + 1] = d.order_xy[2 * p + 1]; }
            else { xy[2 * p] = d.points[3 * (int64_t)p]; xy[2 * p + 1] = d.points[3 * (int64_t)p + 1]; }
        }

        std::vector<int32_t> rootch;
        if (P > 0) {
            std::vector<int64_t> nodes(P);
            std::iota(nodes.begin(), nodes.end(), 0);
            Scratch sc(P);
            LocalTree T;
            const int32_t root = nd(nodes, 0, sc, T);
            // postorder -> fronts (elimination positions in the same order as a sequential run)
            std::vector<int32_t> gid(T.own.size(), -1);
            for (size_t i = 0; i < T.own.size(); i++) {
                std::vector<int32_t> chl;
                for (int c = 0; c < 2; c++) if (T.ch[i][c] >= 0) chl.push_back(gid[T.ch[i][c]]);
                gid[i] = new_front(std::move(T.own[i]), chl);
            }
            rootch.push_back(gid[root]);
        tick("nested dissection");
        }
        std::vector<int64_t> gl;
        for (int q = 0; q < Q; q++) gl.push_back(vT(q));
        for (int k = 0; k < NS; k++) gl.push_back(vS(k));
        if (!gl.empty() || rootch.empty()) new_front(std::move(gl), rootch);
        // boundaries (fronts are in postorder: children precede parents)
        int32_t nf = (int32_t)S.fronts.size();
        std::vector<int64_t> cand;
        for (int32_t f = 0; f < nf; f++) {
            cand.clear();
            int64_t last = -1;
            for (int64_t v : own[f]) last = std::max(last, S.elim_pos[v]);
            for (int64_t v : own[f])
                for (int64_t k = adj_begin[v]; k < adj_begin[v + 1]; k++)
                    if (S.elim_pos[adj[k]] > last) cand.push_back(adj[k]);
            for (int c = 0; c < S.fronts[f].nchild; c++)
                for (int64_t u : bnd[S.fronts[f].child[c]])
                    if (S.elim_pos[u] > last) cand.push_back(u);
            std::sort(cand.begin(), cand.end(), [&](int64_t a, int64_t b) { return S.elim_pos[a] < S.elim_pos[b]; });
            cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
            bnd[f] = cand;
        }
        tick("boundaries");
        // rows and sizes (every rank knows the whole tree)
        std::vector<std::vector<int64_t>> fv(nf);       // vertex list (row order)
        std::vector<std::vector<int32_t>> fvrow(nf);    // local row of each vertex
        for (int32_t f = 0; f < nf; f++) {
            Front &F = S.fronts[f];
            fv[f] = own[f];
            fv[f].insert(fv[f].end(), bnd[f].begin(), bnd[f].end());
            int32_t m = 0, s = 0;
            F.rows_off = (int64_t)S.rows.size();
            for (size_t i = 0; i < fv[f].size(); i++) {
                int64_t v = fv[f][i];
                fvrow[f].push_back(m);
                for (int k = 0; k < S.vdim[v]; k++) S.rows.push_back((int32_t)(S.voff[v] + k));
                m += S.vdim[v];
                if (i < own[f].size()) s += S.vdim[v];
            }
            F.m = m; F.s = s;
            F.owner = 0; F.rhs_bnd = 0;
        }
        auto front_flops = [&](const Front &F) {
            double sd = F.s, ud = F.m - F.s;
            return sd * sd * sd / 3.0 + ud * sd * sd + ud * ud * sd;
        };
        // heights / levels (global: every rank walks the same level sequence)
        int32_t maxh = 0;
        for (int32_t f = 0; f < nf; f++) {
            Front &F = S.fronts[f];
            int32_t h = 0;
            for (int c = 0; c < F.nchild; c++) h = std::max(h, S.fronts[F.child[c]].height + 1);
            F.height = h;
            maxh = std::max(maxh, h);
        }
        S.nlevels = maxh + 1;
        // ---------------- ranks ----------------
        DistPlan &D = S.dist;
        D.rank = rank; D.nranks = nranks;
        {
            std::vector<double> sub(nf, 0.0);              // subtree flops (fronts are in postorder)
            for (int32_t f = 0; f < nf; f++) {
                sub[f] += front_flops(S.fronts[f]);
                if (S.fronts[f].parent >= 0) sub[S.fronts[f].parent] += sub[f];
            }
            std::vector<int32_t> rlo(nf, 0), rhi(nf, nranks);
            for (int32_t f = nf - 1; f >= 0; f--) {        // parents before children
                Front &F = S.fronts[f];
                if (F.parent < 0) { rlo[f] = 0; rhi[f] = nranks; }
                const int32_t lo = rlo[f], hi = rhi[f];
                F.owner = lo;
                if (F.nchild == 2 && hi - lo > 1) {
                    const double a = sub[F.child[0]], b = sub[F.child[1]];
                    int32_t mid = lo + (int32_t)std::lround((double)(hi - lo) * a / std::max(a + b, 1e-300));
                    mid = std::min(std::max(mid, lo + 1), hi - 1);
                    rlo[F.child[0]] = lo; rhi[F.child[0]] = mid;
                    rlo[F.child[1]] = mid; rhi[F.child[1]] = hi;
                } else {
                    for (int c = 0; c < F.nchild; c++) { rlo[F.child[c]] = lo; rhi[F.child[c]] = hi; }
                }
            }
        }
        auto local = [&](int32_t f) { return S.fronts[f].owner == rank; };
        for (int32_t f = 0; f < nf; f++) {
            const Front &F = S.fronts[f];
            if (local(f) && F.parent >= 0 && !local(F.parent)) {
                if (D.top >= 0) { S.error = "internal: two top fronts on one rank"; return false; }
                D.top = f;
            }
        }
        if (D.top >= 0) S.fronts[D.top].rhs_bnd = 1;
        // offsets: arena / inverses for this rank's fronts, solve vectors also for remote children of
        // them (the forward transfer lands there)
        int64_t aoff = 0, voff2 = 0, ioff = 0, poff = 0;
        for (int32_t f = 0; f < nf; f++) {
            Front &F = S.fronts[f];
            const bool loc = local(f);
            const bool needvec = loc || (F.parent >= 0 && local(F.parent));
            const int32_t m = F.m, s = F.s;
            F.arena_off = loc ? aoff : 0;
            F.vec_off = needvec ? voff2 : 0;
            F.inv_off = loc ? ioff : 0;
            F.panel_off = loc ? (int32_t)poff : 0;
            if (loc) poff += (s + kPanel - 1) / kPanel;
            if (loc) aoff += (int64_t)m * m;
            if (needvec) voff2 += m;
            if (loc && s > 0) ioff += (int64_t)((s - 1) / kPanel) * kPanel * kPanel + (int64_t)((s - 1) % kPanel + 1) * ((s - 1) % kPanel + 1);
            const double fl = front_flops(F);
            const int64_t nz = (int64_t)s * (s + 1) / 2 + (int64_t)(m - s) * s;
            D.factor_flops_total += fl;
            D.nnz_factor_total += nz;
            if (loc) { S.factor_flops += fl; S.nnz_factor += nz; }
        }
        S.arena_size = aoff;
        S.vec_size = voff2;
        S.inv_size = ioff;
        S.npanels = poff;
        auto local_row = [&](int32_t f, int64_t v) -> int32_t {
            const auto &L = fv[f];
            int64_t pv = S.elim_pos[v];
            auto it = std::lower_bound(L.begin(), L.end(), pv, [&](int64_t a, int64_t p) { return S.elim_pos[a] < p; });
            if (it == L.end() || *it != v) return -1;
            return fvrow[f][it - L.begin()];
        };
        // bmap
        for (int32_t f = 0; f < nf; f++) {
            Front &F = S.fronts[f];
            F.bmap_off = (int64_t)S.bmap.size();
            if (F.parent < 0) continue;
            for (int64_t v : bnd[f]) {
                int32_t lr = local_row(F.parent, v);
                if (lr < 0) { S.error = "internal: boundary vertex missing in parent front"; return false; }
                for (int k = 0; k < S.vdim[v]; k++) S.bmap.push_back(lr + k);
            }
        }
        // direct assembly: a child adds its final contribution block into the parent from its last
        // trailing-update launch, unless a sibling of the same level (slot 0) does so in that same
        // launch — then this one (slot 1) goes through the extend-add launch after it, so every
        // parent entry is summed in a fixed order.  A child under a remote parent keeps its
        // contribution block (it is packed and sent).
        for (int32_t f = 0; f < nf; f++) {
            Front &F = S.fronts[f];
            F.direct = 0;
            if (F.parent < 0 || F.m == F.s || F.s == 0) continue;
            if (!local(f) || !local(F.parent)) continue;
            const Front &Pf = S.fronts[F.parent];
            bool slot1 = Pf.nchild > 1 && Pf.child[1] == f;
            bool same = Pf.nchild > 1 && S.fronts[Pf.child[0]].height == S.fronts[Pf.child[1]].height &&
                        local(Pf.child[0]);
            F.direct = (slot1 && same) ? 0 : 1;
        }
        S.level_fronts.assign(S.nlevels, {});
        for (int32_t f = 0; f < nf; f++)
            if (local(f)) S.level_fronts[S.fronts[f].height].push_back(f);
        // cross-rank transfers (one per rank > 0 with work): child = that rank's top front
        for (int32_t f = 0; f < nf; f++) {
            const Front &F = S.fronts[f];
            if (F.parent < 0 || S.fronts[F.parent].owner == F.owner || F.m == F.s) continue;
            DistPlan::Xfer x;
            x.child = f; x.parent = F.parent; x.src = F.owner; x.dst = S.fronts[F.parent].owner;
            x.level = S.fronts[F.parent].height; x.u = F.m - F.s;
            D.xfers.push_back(x);
        }
        std::stable_sort(D.xfers.begin(), D.xfers.end(), [](const DistPlan::Xfer &a, const DistPlan::Xfer &b) {
            return a.level < b.level || (a.level == b.level && a.child < b.child);
        });
        for (auto &x : D.xfers)
            if (x.src == rank || x.dst == rank) {
                x.buf_off = D.xbuf_size;
                D.xbuf_size += (int64_t)x.u * (x.u + 1) / 2;
            }
        // edge ownership: the owner of the front of the edge's first-eliminated vertex
        auto first_owner = [&](const int64_t *v, int n) {
            int64_t best = v[0];
            for (int k = 1; k < n; k++) if (S.elim_pos[v[k]] < S.elim_pos[best]) best = v[k];
            return S.fronts[vfront[best]].owner;
        };
        for (int e = 0; e < d.n_rep; e++) {
            int64_t v[1] = {vP(d.rep_point[e])};
            if (first_owner(v, 1) == rank) D.own_rep.push_back(e);
        }
        for (int e = 0; e < d.n_depth; e++) {
            int64_t v[2] = {vP(d.dep_point[e]), vS(d.dep_scale[e])};
            if (first_owner(v, 2) == rank) D.own_dep.push_back(e);
        }
        for (int e = 0; e < d.n_arap; e++) {
            int64_t v[5];
            for (int k = 0; k < 4; k++) v[k] = vP(d.arap_pts[4 * (int64_t)e + k]);
            v[4] = vT(d.arap_pair[e]);
            if (first_owner(v, 5) == rank) D.own_arap.push_back(e);
        }
        D.vertex_owner.resize(S.nv);
        D.dof_local.assign(S.ndof, 0);
        for (int64_t v = 0; v < S.nv; v++) {
            D.vertex_owner[v] = S.fronts[vfront[v]].owner;
            if (D.vertex_owner[v] == rank)
                for (int k = 0; k < S.vdim[v]; k++) D.dof_local[S.voff[v] + k] = 1;
        }
        if (std::getenv("DEFTRI_DEBUG_PLAN")) {
            for (int32_t h = 0; h < S.nlevels; h++) {
                int32_t ms = 0, mm = 0; double fl = 0;
                for (int32_t f : S.level_fronts[h]) {
                    const Front &F = S.fronts[f];
                    ms = std::max(ms, F.s); mm = std::max(mm, F.m);
                    fl += front_flops(F);
                }
                std::fprintf(stderr, "[plan] rank %d level %d fronts %zu max_s %d max_m %d flops %.3g\n", rank, h,
                             S.level_fronts[h].size(), ms, mm, fl);
            }
        }

        tick("fronts/ranks/offsets");
        // ---------------- H blocks ----------------
        // column vertex c, row vertices r with elim[r] >= elim[c], r coupled with c (or r == c).  A
        // column of this rank's fronts: every coupled row (blocks no owned edge feeds stay zero; the
        // other ranks' parts arrive through their contribution blocks).  A remote column in the top
        // front's boundary: the coupled rows inside that front, placed in its contribution-block
        // region (no lambda there: the owner adds it).
        const int32_t X = D.top;
        std::vector<int64_t> blk_begin(S.nv + 1, 0);
        std::vector<int64_t> blk_rowv;
        std::vector<int32_t> blk_front;
        for (int64_t c = 0; c < S.nv; c++) {
            blk_begin[c] = (int64_t)blk_rowv.size();
            int32_t tf = -1;
            if (local(vfront[c])) tf = vfront[c];
            else if (X >= 0 && local_row(X, c) >= 0) tf = X;
            if (tf < 0) continue;
            std::vector<int64_t> rs;
            rs.push_back(c);
            for (int64_t k = adj_begin[c]; k < adj_begin[c + 1]; k++)
                if (S.elim_pos[adj[k]] > S.elim_pos[c] && (tf != X || vfront[c] == X || local_row(X, adj[k]) >= 0))
                    rs.push_back(adj[k]);
            std::sort(rs.begin(), rs.end());
            blk_rowv.insert(blk_rowv.end(), rs.begin(), rs.end());
            blk_front.insert(blk_front.end(), rs.size(), tf);
        }
        blk_begin[S.nv] = (int64_t)blk_rowv.size();
        S.nblocks = (int64_t)blk_rowv.size();
        S.blk_val_off.resize(S.nblocks); S.blk_rows.resize(S.nblocks); S.blk_cols.resize(S.nblocks);
        S.blk_arena.resize(S.nblocks); S.blk_ld.resize(S.nblocks); S.blk_diag.resize(S.nblocks);
        S.blk_row_dof.resize(S.nblocks); S.blk_col_dof.resize(S.nblocks);
        int64_t hv = 0;
        for (int64_t c = 0; c < S.nv; c++) {
            for (int64_t b = blk_begin[c]; b < blk_begin[c + 1]; b++) {
                const int32_t f = blk_front[b];
                const Front &F = S.fronts[f];
                const int32_t lc = local_row(f, c);
                int64_t r = blk_rowv[b];
                int32_t lr = local_row(f, r);
                if (lr < 0 || lc < 0) { S.error = "internal: block outside its front"; return false; }
                S.blk_rows[b] = S.vdim[r]; S.blk_cols[b] = S.vdim[c];
                S.blk_val_off[b] = hv; hv += (int64_t)S.vdim[r] * S.vdim[c];
                S.blk_arena[b] = F.arena_off + (int64_t)lc * F.m + lr;
                S.blk_ld[b] = F.m;
                S.blk_diag[b] = (r == c && f == vfront[c]) ? 1 : 0;
                S.blk_row_dof[b] = S.voff[r];
                S.blk_col_dof[b] = S.voff[c];
            }
        }
        S.hval_size = hv;
        auto block_id = [&](int64_t c, int64_t r) -> int64_t {
            auto b0 = blk_rowv.begin() + blk_begin[c], b1 = blk_rowv.begin() + blk_begin[c + 1];
            auto it = std::lower_bound(b0, b1, r);
            if (it == b1 || *it != r) return -1;
            return it - blk_rowv.begin();
        };
        // contributions
        std::vector<std::pair<int64_t, uint64_t>> hc;      // (block, record)
        std::vector<std::pair<int64_t, uint64_t>> bc;      // (vertex, record)
        hc.reserve(D.own_rep.size() + 3 * D.own_dep.size() + 15 * D.own_arap.size());
        bc.reserve(D.own_rep.size() + 2 * D.own_dep.size() + 5 * D.own_arap.size());
        auto add_edge = [&](int kind, int64_t e, const int64_t *v, int nr) {
            for (int a = 0; a < nr; a++) {
                bc.emplace_back(v[a], contrib_pack(kind, e, a, a));
                for (int b = 0; b < nr; b++) {
                    int64_t c = v[a], r = v[b];
                    if (S.elim_pos[r] < S.elim_pos[c]) continue;
                    if (S.elim_pos[r] == S.elim_pos[c] && r != c) continue;
                    int64_t bid = block_id(c, r);
                    if (bid < 0) { S.error = "internal: missing block"; return false; }
                    hc.emplace_back(bid, contrib_pack(kind, e, a, b));
                }
            }
            return true;
        };
        // owned edges only, numbered in this rank's (compacted) edge arrays
        for (size_t k = 0; k < D.own_rep.size(); k++) {
            const int e = D.own_rep[k];
            int64_t v[1] = {vP(d.rep_point[e])};
            if (!add_edge(EK_REP, (int64_t)k, v, 1)) return false;
        }
        for (size_t k = 0; k < D.own_dep.size(); k++) {
            const int e = D.own_dep[k];
            int64_t v[2] = {vP(d.dep_point[e]), vS(d.dep_scale[e])};
            if (!add_edge(EK_DEP, (int64_t)k, v, 2)) return false;
        }
        for (size_t k = 0; k < D.own_arap.size(); k++) {
            const int e = D.own_arap[k];
            int64_t v[5];
            for (int q = 0; q < 4; q++) v[q] = vP(d.arap_pts[4 * (int64_t)e + q]);
            v[4] = vT(d.arap_pair[e]);
            if (!add_edge(EK_ARAP, (int64_t)k, v, 5)) return false;
        }
        auto chunkify = [&](std::vector<std::pair<int64_t, uint64_t>> &lst, int64_t nkeys,
                            std::vector<uint64_t> &recs, std::vector<int64_t> &cbeg,
                            std::vector<int32_t> &clen, std::vector<int32_t> &ckey,
                            std::vector<int64_t> &key_chunk) {
            // stable counting sort by key (the records of a key keep their edge order)
            std::vector<int64_t> kbeg(nkeys + 1, 0);
            for (const auto &x : lst) kbeg[x.first + 1]++;
            for (int64_t k = 0; k < nkeys; k++) kbeg[k + 1] += kbeg[k];
            recs.resize(lst.size());
            {
                std::vector<int64_t> pos(kbeg.begin(), kbeg.end() - 1);
                for (const auto &x : lst) recs[pos[x.first]++] = x.second;
            }
            std::vector<std::pair<int64_t, uint64_t>>().swap(lst);
            key_chunk.assign(nkeys + 1, 0);
            for (int64_t k = 0; k < nkeys; k++) {
                key_chunk[k] = (int64_t)cbeg.size();
                for (int64_t s0 = kbeg[k]; s0 < kbeg[k + 1]; s0 += kChunk) {
                    cbeg.push_back(s0);
                    clen.push_back((int32_t)std::min<int64_t>(kChunk, kbeg[k + 1] - s0));
                    ckey.push_back((int32_t)k);
                }
            }
            key_chunk[nkeys] = (int64_t)cbeg.size();
        };
        chunkify(hc, S.nblocks, S.hcontrib, S.hchunk_begin, S.hchunk_len, S.hchunk_block, S.hblk_chunk_begin);
        tick("blocks+contributions");
        chunkify(bc, S.nv, S.bcontrib, S.bchunk_begin, S.bchunk_len, S.bchunk_vertex, S.bv_chunk_begin);

        tick("chunking");
        // ---------------- task lists ----------------
        auto push3 = [&](int32_t a, int32_t b, int32_t c) {
            S.task_i32.push_back(a); S.task_i32.push_back(b); S.task_i32.push_back(c);
        };
        S.levels.assign(S.nlevels, {});
        // DEFTRI_TRSM_FUSE=1: the panel TRSM rides the launch that factors the diagonal tile (tail
        // tiles); measured at C2: 12.15 vs 12.36 ms per trial against separate k_trsm launches with the
        // same W publication, but slower than the plain schedule without it (11.8) — off by default
        static const bool trsm_fuse = [] {
            const char *e = std::getenv("DEFTRI_TRSM_FUSE");
            return e && std::atoi(e) == 1;
        }();
        std::unordered_set<int64_t> trsm_fused;             // (front, panel k0) whose TRSM rides an earlier launch
        S.trsm_fused = trsm_fuse;
        for (int32_t h = 0; h < S.nlevels; h++) {
            auto &LT = S.levels[h];
            const auto &fs = S.level_fronts[h];
            for (int slot = 0; slot < 2; slot++) {
                LT.ea_off[slot] = (int64_t)S.task_i32.size() / 3;
                int32_t cnt = 0;
                for (int32_t f : fs) {
                    const Front &F = S.fronts[f];
                    if (F.nchild <= slot) continue;
                    int32_t c = F.child[slot];
                    if (S.fronts[c].direct) continue;           // assembled by its own last update
                    if (!local(c)) continue;                     // another rank's: packed transfer (DistPlan)
                    int32_t u = S.fronts[c].m - S.fronts[c].s;
                    // (child, 16 CB columns j0.., 256 CB rows i0..), lower triangle only
                    for (int32_t j = 0; j < u; j += 16)
                        for (int32_t i = j; i < u; i += 256) { push3(c, j, i); cnt++; }
                }
                LT.nea[slot] = cnt;
            }
            int32_t maxs = 0;
            for (int32_t f : fs) maxs = std::max(maxs, S.fronts[f].s);
            // two-level right-looking schedule.  Outer blocks of kOuter own columns; inside one, each
            // 64-wide panel k0 gets [diag (k0 == 0 only; later panels are factored by the update
            // launch that finishes their diagonal tile)] + trsm + an inner update restricted to the
            // block's remaining own columns; after the block, one outer update with K = the block
            // width covers every trailing column (own and contribution block).
            // update modes: INNER = panel kA's update of the outer block's remaining own columns;
            // FULL = block kA's update of every trailing column; LOOK = the next block's columns only
            // (carries the fused factorization of its first panel); REST = the columns past the next
            // block (and the whole trailing part of fronts that end in this block).
            // OWN = FULL restricted to the front's own trailing columns (carries the fused panel
            // factorization; main stream); CB = FULL restricted to the contribution-block columns (needed
            // only by the parent's assembly at the next level: side stream, overlapping the rest of the
            // level's panel chain).
            enum { UP_INNER = 1, UP_FULL = 0, UP_LOOK = 2, UP_REST = 3, UP_OWN = 4, UP_CB = 5 };
            auto push_update = [&](Symbolic::StepTasks &st, int32_t kA, int32_t kmax, int mode) {
                st.upd_off = (int64_t)S.task_i32.size() / 3;
                st.kA = kA; st.kmax = kmax;
                st.inner = mode == UP_INNER ? 1 : mode == UP_LOOK ? 2 : mode == UP_OWN ? 3 : 0;
                const int32_t Pend = (kA / kOuter + 1) * kOuter;
                // pass 0: the tiles that carry a fused panel factorization go first in the launch
                std::vector<std::array<int32_t, 4>> spans;   // (front, t0 column, tend column, has_diag)
                for (int32_t f : fs) {
                    const Front &F = S.fronts[f];
                    if (F.s <= kA) continue;
                    const int32_t K = std::min(kmax, F.s - kA);
                    int32_t t0 = kA + K, tend = F.m;
                    if (mode == UP_INNER) tend = std::min(F.s, Pend);
                    if (mode == UP_LOOK) { if (F.s <= Pend) continue; t0 = Pend; tend = std::min(F.s, Pend + kOuter); }
                    if (mode == UP_REST && F.s > Pend) t0 = std::min(F.s, Pend + kOuter);
                    if (mode == UP_OWN) tend = F.s;                 // k_update stores c < s only (inner 3)
                    if (mode == UP_CB) t0 = std::max(t0, F.s);
                    if (t0 >= tend) continue;
                    const bool has_diag = (mode == UP_INNER || mode == UP_LOOK || mode == UP_FULL || mode == UP_OWN) &&
                                          F.s > t0 && t0 == kA + K;
                    spans.push_back({f, t0, tend, has_diag ? 1 : 0});
                }
                // pass 1: the other tiles; pass 2 (trsm_fuse): the column tiles below each fused diagonal
                // tile, last in the launch (they wait for that panel's factorization)
                for (int pass = 0; pass < 3; pass++)
                    for (const auto &sp : spans) {
                        const int32_t f = sp[0], t0 = sp[1], tend = sp[2];
                        const bool has_diag = sp[3] != 0;
                        const Front &F = S.fronts[f];
                        if (pass == 0) {
                            if (has_diag) { push3(f, t0, t0); st.nupd++; }
                            continue;
                        }
                        const bool fuse = has_diag && trsm_fuse;
                        if (pass == 2) {
                            if (!fuse) continue;
                            for (int32_t ti = t0 + kPanel; ti < F.m; ti += 64) { push3(f, ti, t0); st.nupd++; st.ntail++; }
                            trsm_fused.insert(((int64_t)f << 32) | (uint32_t)t0);
                            continue;
                        }
                        for (int32_t tj = t0; tj < tend; tj += 64)
                            for (int32_t ti = tj; ti < F.m; ti += 64) {
                                if (has_diag && ti == t0 && tj == t0) continue;
                                if (fuse && tj == t0) continue;
                                push3(f, ti, tj); st.nupd++;
                            }
                    }
                for (const auto &sp : spans) {
                    const Front &F = S.fronts[sp[0]];
                    const int32_t K = std::min(kmax, F.s - kA), t0 = sp[1], tend = sp[2];
                    for (int32_t tj = t0; tj < tend; tj += 64)
                        for (int32_t ti = tj; ti < F.m; ti += 64) {
                            double fl = 2.0 * std::min(64, F.m - ti) * std::min(64, tend - tj) * K;
                            S.update_flops += fl;
                            st.upd_flops += fl;
                        }
                }
            };
            for (int32_t P0 = 0; P0 < maxs; P0 += kOuter) {
                for (int32_t k0 = P0; k0 < std::min(maxs, P0 + kOuter); k0 += kPanel) {
                    Symbolic::StepTasks st;
                    st.k0 = k0;
                    st.diag_off = (int64_t)S.task_i32.size() / 3;
                    for (int32_t f : fs) if (S.fronts[f].s > k0) {
                        if (k0 == 0) { push3(f, k0, 0); st.ndiag++; }
                        double kb = std::min(kPanel, S.fronts[f].s - k0);
                        S.diag_flops += kb * kb * kb / 3.0;
                    }
                    if (k0 == 0 && trsm_fuse)               // the level's first panel: TRSM tiles ride the diag launch
                        for (int32_t f : fs) {
                            const Front &F = S.fronts[f];
                            if (F.s <= 0) continue;
                            for (int32_t r0 = kPanel; r0 < F.m; r0 += 64) {
                                push3(f, 0, r0); st.ndiag_tail++;
                                S.trsm_flops += (double)std::min(64, F.m - r0) * std::min(kPanel, F.s) * std::min(kPanel, F.s);
                            }
                            trsm_fused.insert(((int64_t)f << 32) | 0u);
                        }
                    st.trsm_off = (int64_t)S.task_i32.size() / 3;
                    for (int32_t f : fs) {
                        const Front &F = S.fronts[f];
                        if (F.s <= k0) continue;
                        if (trsm_fused.count(((int64_t)f << 32) | (uint32_t)k0)) {
                            const int32_t kb = std::min(kPanel, F.s - k0);
                            for (int32_t r0 = k0 + kPanel; r0 < F.m; r0 += 64) S.trsm_flops += (double)std::min(64, F.m - r0) * kb * kb;
                            continue;
                        }
                        int32_t kb = std::min(kPanel, F.s - k0);
                        for (int32_t r0 = k0 + kb; r0 < F.m; r0 += 64) {
                            push3(f, k0, r0); st.ntrsm++;
                            S.trsm_flops += (double)std::min(64, F.m - r0) * kb * kb;
                        }
                    }
                    push_update(st, k0, kPanel, UP_INNER);
                    LT.steps.push_back(st);
                }
                // outer update of block P0: when some front continues past the block, split it into
                // REST (side stream, overlaps the next block's panel chain) and LOOK (main stream: the
                // next block's columns + the fused factorization of its first panel)
                // Measured at C2 on MI355X: the split (one more launch per block) costs more than the
                // overlap recovers (19.2 vs 18.9 LM it/s), so it is off unless DEFTRI_LOOKAHEAD_MIN_M
                // names the smallest front order that should use it.
                const char *la_env = std::getenv("DEFTRI_LOOKAHEAD_MIN_M");
                const int32_t la_min_m = la_env ? std::atoi(la_env) : std::numeric_limits<int32_t>::max();
                bool cont = false;
                int32_t maxm = 0;
                for (int32_t f : fs) { cont = cont || S.fronts[f].s > P0 + kOuter; maxm = std::max(maxm, S.fronts[f].m); }
                const bool cont_any = cont;
                cont = cont && maxm >= la_min_m;
                auto outer_step = [&](int mode, int stream, int wait_side) {
                    Symbolic::StepTasks so;
                    so.k0 = P0;
                    so.diag_off = so.trsm_off = (int64_t)S.task_i32.size() / 3;
                    push_update(so, P0, kOuter, mode);
                    so.stream = stream; so.wait_side = wait_side;
                    LT.steps.push_back(so);
                };
                // (the contribution-block update first on the side stream, the OWN update concurrently
                // on the main stream: measured at C2 slower — side-stream contention)
                (void)cont_any;
                if (cont) {
                    outer_step(UP_REST, 1, 0);
                    outer_step(UP_LOOK, 0, 1);
                } else {
                    // touches the trailing columns an earlier REST (side stream) may still be updating
                    outer_step(UP_FULL, 0, 2);
                }
            }
            LT.fwd_off = (int64_t)S.task_i32.size() / 3;
            for (int32_t f : fs) { push3(f, 0, 0); LT.nfwd++; }
            for (int32_t k0 = 0; k0 < maxs; k0 += kPanel) {
                Symbolic::LevelTasks::SolveStep st;
                st.off = (int64_t)S.task_i32.size() / 3;
                for (int32_t f : fs) {
                    const Front &F = S.fronts[f];
                    if (F.s <= k0) continue;
                    int32_t kb = std::min(kPanel, F.s - k0);
                    push3(f, k0, k0); st.n++;
                    for (int32_t r0 = k0 + kb; r0 < F.m; r0 += 64) { push3(f, k0, r0); st.n++; }
                }
                LT.fsteps.push_back(st);
            }
            LT.fchain_off = (int64_t)S.task_i32.size() / 3;
            for (int32_t f : fs) {
                const Front &F = S.fronts[f];
                for (int32_t r0 = 0; r0 < F.m; r0 += 64) { push3(f, r0, 0); LT.nfchain++; }
            }
            LT.bchain_off = (int64_t)S.task_i32.size() / 3;
            for (int32_t f : fs) {
                const Front &F = S.fronts[f];
                if (F.s <= 0) continue;
                for (int32_t c0 = ((F.s - 1) / 64) * 64; c0 >= 0; c0 -= 64) { push3(f, c0, 0); LT.nbchain++; }
            }
            LT.bgemv_off = (int64_t)S.task_i32.size() / 3;
            for (int32_t f : fs) {
                const Front &F = S.fronts[f];
                for (int32_t c0 = 0; c0 < F.s; c0 += kBwdCols) { push3(f, c0, 0); LT.nbgemv++; }
            }
            int32_t npan = (maxs + kPanel - 1) / kPanel;
            for (int32_t p = npan - 1; p >= 0; p--) {
                int32_t k0 = p * kPanel;
                Symbolic::LevelTasks::SolveStep st;
                st.off = (int64_t)S.task_i32.size() / 3;
                for (int32_t f : fs) {
                    const Front &F = S.fronts[f];
                    if (F.s <= k0) continue;
                    push3(f, k0, k0); st.n++;
                    for (int32_t q0 = 0; q0 < k0; q0 += 64) { push3(f, k0, q0); st.n++; }
                }
                LT.bsteps.push_back(st);
            }
        }
        tick("task lists");
        // packed extend-add of the contribution blocks received from other ranks (same task shape as
        // the extend-add: 16 CB columns x 256 CB rows, lower triangle)
        for (auto &x : D.xfers) {
            if (x.dst != rank) continue;
            x.ea_off = (int64_t)S.task_i32.size() / 3;
            for (int32_t j = 0; j < x.u; j += 16)
                for (int32_t i = j; i < x.u; i += 256) { push3(x.child, j, i); x.nea++; }
        }
        return true;
    }
};

}  // namespace

bool analyse(const deftri_problem_desc &d, Symbolic &S, int leaf_points, int rank, int nranks) {
    S = Symbolic();
    if (nranks < 1 || rank < 0 || rank >= nranks) { S.error = "bad rank / nranks"; return false; }
    Builder b(d, S, leaf_points, rank, nranks);
    const bool ok = b.run();
    if (const char *path = std::getenv("DEFTRI_DUMP_FRONTS"); ok && path) {   // plan inspection (tools/)
        if (FILE *fp = std::fopen(path, "w")) {
            for (int32_t h = 0; h < S.nlevels; h++)
                for (int32_t f : S.level_fronts[h])
                    std::fprintf(fp, "%d %d %d %d %d\n", h, f, S.fronts[f].m, S.fronts[f].s, S.fronts[f].parent);
            std::fclose(fp);
        }
    }
    return ok;
}

}  // namespace deftri
