// plan_check.cpp — TEST-ONLY host emulation of the multifrontal plan.
//
// Executes the exact task lists that kernels.hip launches (extend-add, panel LDL^T, TRSM,
// trailing update, forward/backward substitution) with plain loops on a dense H supplied by the
// caller.  It exists so the symbolic analysis (ordering, boundary sets, child->parent maps, arena
// offsets, task lists) can be verified in the CPU test suite without a GPU.  It is never called by
// the solve path (deftri_solve_lm et al. run only on the device) — see DESIGN.md §3.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "symbolic.h"

namespace deftri {

// xfer (point-sharded plan only): op 2 send / 3 receive n doubles to / from `peer` (the transport
// of deftri_dist_set_transport).  bpart: the rank's partial b, injected on its top front's boundary.
int plan_emulate_solve(const Symbolic &S, const double *H, double lambda, const double *rhs, double *x,
                       const std::function<int(int, int, double *, int64_t)> *xfer, const double *bpart) {
    const int64_t n = S.ndof;
    const DistPlan &D = S.dist;
    std::vector<double> arena((size_t)S.arena_size, 0.0), vec((size_t)S.vec_size, 0.0);
    // scatter: every block entry from the dense H (row-major n x n)
    int32_t nf = (int32_t)S.fronts.size();
    std::vector<std::pair<int64_t, int32_t>> starts;       // this rank's fronts by arena offset
    for (int32_t f = 0; f < nf; f++)
        if (S.fronts[f].owner == D.rank) starts.emplace_back(S.fronts[f].arena_off, f);
    std::sort(starts.begin(), starts.end());
    for (int64_t b = 0; b < S.nblocks; b++) {
        int64_t a = S.blk_arena[b];
        auto it = std::upper_bound(starts.begin(), starts.end(), std::make_pair(a, (int32_t)nf));
        const int32_t f = (it - 1)->second;
        const Front &F = S.fronts[f];
        int32_t lc = (int32_t)((a - F.arena_off) / F.m), lr = (int32_t)((a - F.arena_off) % F.m);
        for (int i = 0; i < S.blk_rows[b]; i++)
            for (int j = 0; j < S.blk_cols[b]; j++) {
                int64_t rdof = S.rows[F.rows_off + lr + i], cdof = S.rows[F.rows_off + lc + j];
                double v = H[rdof * n + cdof] + ((S.blk_diag[b] && i == j) ? lambda : 0.0);
                arena[a + (int64_t)j * F.m + i] = v;
            }
    }
    auto Fp = [&](int32_t f) { return arena.data() + S.fronts[f].arena_off; };
    const int32_t *T = S.task_i32.data();
    if (std::getenv("DEFTRI_DEBUG_EMU")) {
        int64_t nd = 0, nl = 0;
        for (int64_t b = 0; b < S.nblocks; b++) if (S.blk_diag[b]) { nd++; nl += S.blk_cols[b]; }
        int64_t nown = 0;
        for (auto v : D.dof_local) nown += v;
        std::fprintf(stderr, "[emu] rank %d blocks %lld diag blocks %lld lambda dofs %lld own dofs %lld top %d xfers %zu\n",
                     D.rank, (long long)S.nblocks, (long long)nd, (long long)nl, (long long)nown, D.top, D.xfers.size());
        for (const auto &xf : D.xfers) std::fprintf(stderr, "[emu]   xfer child %d parent %d %d->%d level %d u %d\n", xf.child, xf.parent, xf.src, xf.dst, xf.level, xf.u);
        for (int32_t f = 0; f < nf; f++) if (S.fronts[f].parent < 0 || S.fronts[f].height >= S.nlevels - 3)
            std::fprintf(stderr, "[emu]   front %d m %d s %d owner %d parent %d h %d direct %d\n", f, S.fronts[f].m, S.fronts[f].s, S.fronts[f].owner, S.fronts[f].parent, S.fronts[f].height, S.fronts[f].direct);
    }
    auto diag = [&](int f, int k0) -> bool {
        const Front &F = S.fronts[f];
        double *A = Fp(f);
        // kb pivots; in the fused-TRSM plan rows kb..mt-1 of the 64-row diagonal tile become L21 too
        int kb = std::min(64, F.s - k0), m = F.m, mt = S.trsm_fused ? std::min(64, F.m - k0) : kb;
        for (int j = 0; j < kb; j++) {
            double d = A[(int64_t)(k0 + j) * m + k0 + j];
            if (d == 0.0) return false;
            for (int i = j + 1; i < mt; i++) A[(int64_t)(k0 + j) * m + k0 + i] /= d;
            for (int c = j + 1; c < kb; c++)
                for (int i = c; i < mt; i++)
                    A[(int64_t)(k0 + c) * m + k0 + i] -= A[(int64_t)(k0 + j) * m + k0 + i] * d * A[(int64_t)(k0 + j) * m + k0 + c];
        }
        return true;
    };
    // the DistPlan transfers of one level (global order; this rank's part)
    auto level_xfers = [&](int32_t h) {
        std::vector<const DistPlan::Xfer *> v;
        for (const auto &xf : D.xfers)
            if (xf.level == h && (xf.src == D.rank || xf.dst == D.rank)) v.push_back(&xf);
        return v;
    };
    for (int32_t h = 0; h < (int32_t)S.levels.size(); h++) {
        const auto &lv = S.levels[h];
        for (const auto *xf : level_xfers(h)) {                 // packed contribution blocks (k_pack_cb / k_ea_packed)
            const Front &C = S.fronts[xf->child];
            const int u = xf->u;
            std::vector<double> buf((size_t)u * (u + 1) / 2);
            if (xf->src == D.rank) {
                for (int j = 0, o = 0; j < u; j++)
                    for (int i = j; i < u; i++) buf[o++] = Fp(xf->child)[(int64_t)(C.s + j) * C.m + C.s + i];
                if ((*xfer)(2, xf->dst, buf.data(), (int64_t)buf.size())) return -2;
            } else {
                if ((*xfer)(3, xf->src, buf.data(), (int64_t)buf.size())) return -2;
                const Front &Pf = S.fronts[C.parent];
                const int32_t *bm = S.bmap.data() + C.bmap_off;
                for (int j = 0, o = 0; j < u; j++)
                    for (int i = j; i < u; i++) Fp(C.parent)[(int64_t)bm[j] * Pf.m + bm[i]] += buf[o++];
            }
        }
        for (int slot = 0; slot < 2; slot++)
            for (int32_t t = 0; t < lv.nea[slot]; t++) {
                const int32_t *tk = T + 3 * (lv.ea_off[slot] + t);
                int c = tk[0], j0 = tk[1], i0 = tk[2];
                const Front &C = S.fronts[c];
                const Front &Pf = S.fronts[C.parent];
                int u = C.m - C.s;
                const int32_t *bm = S.bmap.data() + C.bmap_off;
                for (int j = j0; j < std::min(j0 + 16, u); j++)
                    for (int i = std::max(j, i0); i < std::min(i0 + 256, u); i++)
                        Fp(C.parent)[(int64_t)bm[j] * Pf.m + bm[i]] += Fp(c)[(int64_t)(C.s + j) * C.m + C.s + i];
            }
        // rows r0..r0+63 of panel k0: L = A L11^{-T} D^{-1} (k_trsm / the fused TRSM tiles)
        auto trsm = [&](int f, int k0, int r0) {
            const Front &F = S.fronts[f];
            double *A = Fp(f);
            int kb = std::min(64, F.s - k0), m = F.m;
            for (int i = r0; i < std::min(r0 + 64, m); i++) {
                double z[64];
                for (int j = 0; j < kb; j++) {
                    double v = A[(int64_t)(k0 + j) * m + i];
                    for (int c = 0; c < j; c++) v -= A[(int64_t)(k0 + c) * m + k0 + j] * z[c];
                    z[j] = v;
                }
                for (int j = 0; j < kb; j++) A[(int64_t)(k0 + j) * m + i] = z[j] / A[(int64_t)(k0 + j) * m + k0 + j];
            }
        };
        for (const auto &st : lv.steps) {
            for (int32_t t = 0; t < st.ndiag; t++) {
                const int32_t *tk = T + 3 * (st.diag_off + t);
                if (!diag(tk[0], tk[1])) return -1;
            }
            for (int32_t t = st.ndiag; t < st.ndiag + st.ndiag_tail; t++) {      // fused TRSM tiles of the diag launch
                const int32_t *tk = T + 3 * (st.diag_off + t);
                trsm(tk[0], tk[1], tk[2]);
            }
            for (int32_t t = 0; t < st.ntrsm; t++) {
                const int32_t *tk = T + 3 * (st.trsm_off + t);
                trsm(tk[0], tk[1], tk[2]);
            }
            for (int32_t t = 0; t < st.nupd; t++) {
                const int32_t *tk = T + 3 * (st.upd_off + t);
                int f = tk[0], ti = tk[1], tj = tk[2];
                const Front &F = S.fronts[f];
                double *A = Fp(f);
                int k0 = st.kA, kb = std::min(st.kmax, F.s - k0), m = F.m;
                int cend = st.inner == 1 ? std::min(F.s, (k0 / kOuter + 1) * kOuter)
                         : st.inner == 2 ? std::min(F.s, (k0 / kOuter + 2) * kOuter)
                         : st.inner == 3 ? F.s : m;
                for (int c = tj; c < std::min(tj + 64, cend); c++)
                    for (int r = ti; r < std::min(ti + 64, m); r++) {
                        double acc = 0;
                        for (int k = 0; k < kb; k++)
                            acc += A[(int64_t)(k0 + k) * m + r] * (A[(int64_t)(k0 + k) * m + c] * A[(int64_t)(k0 + k) * m + k0 + k]);
                        A[(int64_t)c * m + r] -= acc;
                    }
                // direct assembly (k_update): the front's final contribution block goes to the parent
                if (!st.inner && k0 + kb == F.s && F.direct) {
                    const Front &Pf = S.fronts[F.parent];
                    const int32_t *bm = S.bmap.data() + F.bmap_off - F.s;
                    for (int c = tj; c < std::min(tj + 64, m); c++)
                        for (int r = std::max(ti, c); r < std::min(ti + 64, m); r++)
                            Fp(F.parent)[(int64_t)bm[c] * Pf.m + bm[r]] += A[(int64_t)c * m + r];
                }
            }
            // fused panel factorization of the next panel (k_update on the diagonal tile)
            for (int32_t t = 0; t < st.nupd; t++) {
                const int32_t *tk = T + 3 * (st.upd_off + t);
                const Front &F = S.fronts[tk[0]];
                int k1 = st.kA + std::min(st.kmax, F.s - st.kA);
                if (tk[1] == tk[2] && tk[1] == k1 && F.s > k1 && !diag(tk[0], k1)) return -1;
            }
            // fused TRSM tiles: the launch's last ntail tasks (ti, k1) solve their rows once k1 is factored
            for (int32_t t = st.nupd - st.ntail; t < st.nupd; t++) {
                const int32_t *tk = T + 3 * (st.upd_off + t);
                trsm(tk[0], tk[2], tk[1]);
            }
        }
    }
    // forward: gather, then panel steps (same task semantics as k_fwd_gather / k_fwd_step)
    std::vector<double> yv((size_t)S.vec_size, 0.0);
    auto lower_solve = [&](const Front &F, const double *A, int k0, int kb, const double *b, double *y) {
        for (int i = 0; i < kb; i++) y[i] = b[i];
        for (int j = 0; j < kb; j++)
            for (int i = j + 1; i < kb; i++) y[i] -= A[(int64_t)(k0 + j) * F.m + k0 + i] * y[j];
    };
    for (int32_t h = 0; h < (int32_t)S.levels.size(); h++) {
        const auto &lv = S.levels[h];
        for (const auto *xf : level_xfers(h)) {                 // forward-update vectors
            const Front &C = S.fronts[xf->child];
            double *v = vec.data() + C.vec_off + C.s;
            if ((*xfer)(xf->src == D.rank ? 2 : 3, xf->src == D.rank ? xf->dst : xf->src, v, xf->u)) return -2;
        }
        for (int32_t t = 0; t < lv.nfwd; t++) {
            int f = T[3 * (lv.fwd_off + t)];
            const Front &F = S.fronts[f];
            double *v = vec.data() + F.vec_off;
            const int32_t *rows = S.rows.data() + F.rows_off;
            const bool inject = bpart && F.rhs_bnd;
            for (int r = 0; r < F.m; r++) v[r] = r < F.s ? rhs[rows[r]] : (inject ? bpart[rows[r]] : 0.0);
            for (int sl = 0; sl < F.nchild; sl++) {
                const Front &C = S.fronts[F.child[sl]];
                const int32_t *bm = S.bmap.data() + C.bmap_off;
                for (int i = 0; i < C.m - C.s; i++) v[bm[i]] += vec[C.vec_off + C.s + i];
            }
        }
        for (const auto &sp : lv.fsteps) {
            // all tasks of a step read the panel rows before any task writes (device: one launch)
            std::vector<std::vector<double>> ys(sp.n);
            for (int32_t t = 0; t < sp.n; t++) {
                const int32_t *tk = T + 3 * (sp.off + t);
                const Front &F = S.fronts[tk[0]];
                int k0 = tk[1], kb = std::min(64, F.s - k0);
                ys[t].resize(kb);
                lower_solve(F, Fp(tk[0]), k0, kb, vec.data() + F.vec_off + k0, ys[t].data());
            }
            for (int32_t t = 0; t < sp.n; t++) {
                const int32_t *tk = T + 3 * (sp.off + t);
                const Front &F = S.fronts[tk[0]];
                const double *A = Fp(tk[0]);
                int k0 = tk[1], r0 = tk[2], kb = std::min(64, F.s - k0);
                if (r0 == k0) {
                    for (int i = 0; i < kb; i++) yv[F.vec_off + k0 + i] = ys[t][i];
                    continue;
                }
                for (int r = r0; r < std::min(r0 + 64, F.m); r++) {
                    double acc = 0;
                    for (int c = 0; c < kb; c++) acc += A[(int64_t)(k0 + c) * F.m + r] * ys[t][c];
                    vec[F.vec_off + r] -= acc;
                }
            }
        }
    }
    std::memset(x, 0, sizeof(double) * (size_t)n);
    for (size_t hh = S.levels.size(); hh-- > 0;) {
        const auto &lv = S.levels[hh];
        for (int32_t t = 0; t < lv.nbgemv; t++) {
            const int32_t *tk = T + 3 * (lv.bgemv_off + t);
            const Front &F = S.fronts[tk[0]];
            const double *A = Fp(tk[0]);
            const int32_t *rows = S.rows.data() + F.rows_off;
            for (int c = tk[1]; c < std::min(tk[1] + kBwdCols, F.s); c++) {
                double acc = 0;
                for (int i = F.s; i < F.m; i++) acc += A[(int64_t)c * F.m + i] * x[rows[i]];
                vec[F.vec_off + c] = yv[F.vec_off + c] / A[(int64_t)c * F.m + c] - acc;
            }
        }
        for (const auto &sp : lv.bsteps) {
            std::vector<std::vector<double>> xs(sp.n);
            for (int32_t t = 0; t < sp.n; t++) {
                const int32_t *tk = T + 3 * (sp.off + t);
                const Front &F = S.fronts[tk[0]];
                const double *A = Fp(tk[0]);
                int k0 = tk[1], kb = std::min(64, F.s - k0);
                std::vector<double> &xp = xs[t];
                xp.assign(vec.begin() + F.vec_off + k0, vec.begin() + F.vec_off + k0 + kb);
                for (int j = kb - 1; j >= 0; j--)
                    for (int i = 0; i < j; i++) xp[i] -= A[(int64_t)(k0 + i) * F.m + k0 + j] * xp[j];
            }
            for (int32_t t = 0; t < sp.n; t++) {
                const int32_t *tk = T + 3 * (sp.off + t);
                const Front &F = S.fronts[tk[0]];
                const double *A = Fp(tk[0]);
                int k0 = tk[1], q0 = tk[2], kb = std::min(64, F.s - k0);
                if (q0 == k0) {
                    const int32_t *rows = S.rows.data() + F.rows_off;
                    for (int i = 0; i < kb; i++) x[rows[k0 + i]] = xs[t][i];
                    continue;
                }
                for (int q = q0; q < q0 + 64; q++) {
                    double acc = 0;
                    for (int i = 0; i < kb; i++) acc += A[(int64_t)q * F.m + k0 + i] * xs[t][i];
                    vec[F.vec_off + q] -= acc;
                }
            }
        }
        for (const auto *xf : level_xfers((int32_t)hh)) {        // boundary solutions down
            const Front &C = S.fronts[xf->child];
            const int32_t *rows = S.rows.data() + C.rows_off + C.s;
            std::vector<double> buf((size_t)xf->u);
            if (xf->dst == D.rank) {
                for (int i = 0; i < xf->u; i++) buf[i] = x[rows[i]];
                if ((*xfer)(2, xf->src, buf.data(), xf->u)) return -2;
            } else {
                if ((*xfer)(3, xf->dst, buf.data(), xf->u)) return -2;
                for (int i = 0; i < xf->u; i++) x[rows[i]] = buf[i];
            }
        }
    }
    return 0;
}

}  // namespace deftri
