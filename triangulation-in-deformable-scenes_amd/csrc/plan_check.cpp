// plan_check.cpp — TEST-ONLY host emulation of the multifrontal plan.
//
// Executes the exact task lists that kernels.hip launches (extend-add, panel LDL^T, TRSM,
// trailing update, forward/backward substitution) with plain loops on a dense H supplied by the
// caller.  It exists so the symbolic analysis (ordering, boundary sets, child->parent maps, arena
// offsets, task lists) can be verified in the CPU test suite without a GPU.  It is never called by
// the solve path (deftri_solve_lm et al. run only on the device) — see DESIGN.md §3.
#include <cmath>
#include <cstring>
#include <vector>

#include "symbolic.h"

namespace deftri {

int plan_emulate_solve(const Symbolic &S, const double *H, double lambda, const double *rhs, double *x) {
    const int64_t n = S.ndof;
    std::vector<double> arena((size_t)S.arena_size, 0.0), vec((size_t)S.vec_size, 0.0);
    // scatter: every block entry from the dense H (row-major n x n)
    int32_t nf = (int32_t)S.fronts.size();
    for (int64_t b = 0; b < S.nblocks; b++) {
        int64_t a = S.blk_arena[b];
        int32_t f = 0;
        {
            int32_t lo = 0, hi = nf - 1;
            while (lo < hi) {
                int32_t mid = (lo + hi + 1) / 2;
                if (S.fronts[mid].arena_off <= a) lo = mid; else hi = mid - 1;
            }
            f = lo;
        }
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
    for (const auto &lv : S.levels) {
        for (int slot = 0; slot < 2; slot++)
            for (int32_t t = 0; t < lv.nea[slot]; t++) {
                const int32_t *tk = T + 3 * (lv.ea_off[slot] + t);
                int c = tk[0], j0 = tk[1];
                const Front &C = S.fronts[c];
                const Front &Pf = S.fronts[C.parent];
                int u = C.m - C.s;
                const int32_t *bm = S.bmap.data() + C.bmap_off;
                for (int j = j0; j < std::min(j0 + 16, u); j++)
                    for (int i = j; i < u; i++)
                        Fp(C.parent)[(int64_t)bm[j] * Pf.m + bm[i]] += Fp(c)[(int64_t)(C.s + j) * C.m + C.s + i];
            }
        for (const auto &st : lv.steps) {
            for (int32_t t = 0; t < st.ndiag; t++) {
                const int32_t *tk = T + 3 * (st.diag_off + t);
                int f = tk[0], k0 = tk[1];
                const Front &F = S.fronts[f];
                double *A = Fp(f);
                int kb = std::min(64, F.s - k0), m = F.m;
                for (int j = 0; j < kb; j++) {
                    double d = A[(int64_t)(k0 + j) * m + k0 + j];
                    if (d == 0.0) return -1;
                    for (int i = j + 1; i < kb; i++) A[(int64_t)(k0 + j) * m + k0 + i] /= d;
                    for (int c = j + 1; c < kb; c++)
                        for (int i = c; i < kb; i++)
                            A[(int64_t)(k0 + c) * m + k0 + i] -= A[(int64_t)(k0 + j) * m + k0 + i] * d * A[(int64_t)(k0 + j) * m + k0 + c];
                }
            }
            for (int32_t t = 0; t < st.ntrsm; t++) {
                const int32_t *tk = T + 3 * (st.trsm_off + t);
                int f = tk[0], k0 = tk[1], r0 = tk[2];
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
            }
            for (int32_t t = 0; t < st.nupd; t++) {
                const int32_t *tk = T + 3 * (st.upd_off + t);
                int f = tk[0], ti = tk[1], tj = tk[2];
                const Front &F = S.fronts[f];
                double *A = Fp(f);
                int k0 = st.k0, kb = std::min(64, F.s - k0), m = F.m;
                for (int c = tj; c < std::min(tj + 64, m); c++)
                    for (int r = ti; r < std::min(ti + 64, m); r++) {
                        double acc = 0;
                        for (int k = 0; k < kb; k++)
                            acc += A[(int64_t)(k0 + k) * m + r] * (A[(int64_t)(k0 + k) * m + c] * A[(int64_t)(k0 + k) * m + k0 + k]);
                        A[(int64_t)c * m + r] -= acc;
                    }
            }
        }
    }
    // forward
    for (const auto &lv : S.levels) {
        for (int32_t t = 0; t < lv.nfwd; t++) {
            int f = T[3 * (lv.fwd_off + t)];
            const Front &F = S.fronts[f];
            const double *A = Fp(f);
            double *v = vec.data() + F.vec_off;
            const int32_t *rows = S.rows.data() + F.rows_off;
            for (int r = 0; r < F.m; r++) v[r] = r < F.s ? rhs[rows[r]] : 0.0;
            for (int sl = 0; sl < F.nchild; sl++) {
                const Front &C = S.fronts[F.child[sl]];
                const int32_t *bm = S.bmap.data() + C.bmap_off;
                for (int i = 0; i < C.m - C.s; i++) v[bm[i]] += vec[C.vec_off + C.s + i];
            }
            for (int j = 0; j < F.s; j++)
                for (int i = j + 1; i < F.s; i++) v[i] -= A[(int64_t)j * F.m + i] * v[j];
        }
        for (int32_t t = 0; t < lv.ngemv; t++) {
            const int32_t *tk = T + 3 * (lv.gemv_off + t);
            const Front &F = S.fronts[tk[0]];
            const double *A = Fp(tk[0]);
            double *v = vec.data() + F.vec_off;
            for (int i = tk[1]; i < std::min(tk[1] + 64, F.m); i++) {
                double acc = 0;
                for (int c = 0; c < F.s; c++) acc += A[(int64_t)c * F.m + i] * v[c];
                v[i] -= acc;
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
            double *v = vec.data() + F.vec_off;
            const int32_t *rows = S.rows.data() + F.rows_off;
            for (int c = tk[1]; c < std::min(tk[1] + 64, F.s); c++) {
                double acc = 0;
                for (int i = F.s; i < F.m; i++) acc += A[(int64_t)c * F.m + i] * x[rows[i]];
                v[c] = v[c] / A[(int64_t)c * F.m + c] - acc;
            }
        }
        for (int32_t t = 0; t < lv.nfwd; t++) {
            int f = T[3 * (lv.fwd_off + t)];
            const Front &F = S.fronts[f];
            const double *A = Fp(f);
            double *v = vec.data() + F.vec_off;
            const int32_t *rows = S.rows.data() + F.rows_off;
            for (int j = F.s - 1; j >= 0; j--) {
                double acc = v[j];
                for (int i = j + 1; i < F.s; i++) acc -= A[(int64_t)j * F.m + i] * v[i];
                v[j] = acc;
            }
            for (int r = 0; r < F.s; r++) x[rows[r]] = v[r];
        }
    }
    return 0;
}

}  // namespace deftri
