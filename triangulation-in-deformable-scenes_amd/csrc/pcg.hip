// pcg.hip — block-Jacobi preconditioned conjugate gradients for the LM step (H + lambda I) dx = b.
//
// Replaces (reference / g2o): the linear solve inside OptimizationAlgorithmLevenberg::solve
// (BlockSolver::solve -> LinearSolverEigen SimplicialLDLT::solve, g2oBundleAdjustment.cc:640-954's
// optimizer) with the iterative step the north star names; the multifrontal LDL^T (kernels.hip)
// stays as the exact fallback the host switches to when an iteration budget runs out or CG breaks
// down.  Preconditioner: one block per vertex (6x6 T_g, 1x1 scale, 3x3 point) of H + lambda I,
// inverted through its Cholesky factor once per trial.
//
// One iteration = two launches:
//   product (it): every workgroup re-sums the previous update's (r.z, r.r) partials in a fixed order,
//                 tests ||r||^2 <= tol^2 ||b||^2 (all workgroups reach the same verdict, so a
//                 converged solve makes the remaining launches return at once), forms
//                 p = z + beta p_prev on the fly and computes q = (H + lambda I) p by row gathers;
//                 partial p.q per workgroup.
//   update (it):  p.q from the partials (+ the heavy rows' chunk sums, in chunk order), alpha,
//                 x += alpha p, r -= alpha q, z = M r, partial (r.z, r.r).
// Every reduction is a fixed-order tree: repeated solves are bit-identical.  HBM traffic per
// iteration at C2 (100k x 2 views): the blocks twice (both orientations of the off-diagonal ones),
// the 16-byte entries, and ~10 dof vectors.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "kernels.h"
#include "pcg.h"

// launch shape of the product (A/B builds: make PCG_WPE=.. PCG_BATCH=..)
#ifndef DEFTRI_PCG_WPE
#define DEFTRI_PCG_WPE 4
#endif
#ifndef DEFTRI_PCG_BATCH
#define DEFTRI_PCG_BATCH 1
#endif

namespace deftri {
namespace dev {

__device__ __forceinline__ PcgEnt load_ent(const PcgEnt *__restrict__ ent, int64_t e) {
    const int4 w = reinterpret_cast<const int4 *>(ent)[e];
    PcgEnt E;
    E.val_off = (int64_t)(uint32_t)w.x | ((int64_t)w.y << 32);
    E.odof = w.z;
    E.odim = (int16_t)(w.w & 0xffff);
    E.tr = (int16_t)(w.w >> 16);
    return E;
}

// p of a dof, formed where it is read: z + beta p_prev (one fma everywhere, so every reader agrees)
__device__ __forceinline__ double pval(const double *__restrict__ zp, double beta, int64_t i) {
    const double2 v = reinterpret_cast<const double2 *>(zp)[i];
    return __fma_rn(beta, v.y, v.x);
}

// acc[0..d) += B p_other for one entry of the row (B the block in this row's orientation)
__device__ __forceinline__ void ent_acc(const PcgEnt &E, int d, const double *__restrict__ hval,
                                        const double *__restrict__ zp, double beta, double acc[6]) {
    const double *h = hval + E.val_off;
    const int od = E.odim;
    double pj[6];
#pragma unroll
    for (int j = 0; j < 6; j++) pj[j] = j < od ? pval(zp, beta, E.odof + j) : 0.0;
    if (!E.tr) {
#pragma unroll
        for (int i = 0; i < 6; i++)
            if (i < d)
#pragma unroll
                for (int j = 0; j < 6; j++)
                    if (j < od) acc[i] += h[i * od + j] * pj[j];
    } else {
#pragma unroll
        for (int i = 0; i < 6; i++)
            if (i < d)
#pragma unroll
                for (int j = 0; j < 6; j++)
                    if (j < od) acc[i] += h[j * d + i] * pj[j];
    }
}

// fixed-order workgroup sums: thread t adds part[t], part[t + 256], ... then a fixed LDS tree
__device__ __forceinline__ double wg_tree(double a, double *red) {
    red[threadIdx.x] = a;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    const double s = red[0];
    __syncthreads();
    return s;
}

__device__ __forceinline__ void wg_sum2(const double *__restrict__ part, int n, double &s0, double &s1,
                                        double (*red)[256]) {
    double a0 = 0.0, a1 = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) { a0 += part[2 * i]; a1 += part[2 * i + 1]; }
    red[0][threadIdx.x] = a0;
    red[1][threadIdx.x] = a1;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) {
            red[0][threadIdx.x] += red[0][threadIdx.x + off];
            red[1][threadIdx.x] += red[1][threadIdx.x + off];
        }
        __syncthreads();
    }
    s0 = red[0][0];
    s1 = red[1][0];
    __syncthreads();
}

__device__ __forceinline__ void wg_pair_tree(double a0, double a1, double (*red)[256], double *out) {
    red[0][threadIdx.x] = a0;
    red[1][threadIdx.x] = a1;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) {
            red[0][threadIdx.x] += red[0][threadIdx.x + off];
            red[1][threadIdx.x] += red[1][threadIdx.x + off];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) { out[0] = red[0][0]; out[1] = red[1][0]; }
}

// one heavy slot of a slice (heavy vertex of dimension OD): the row side acc += B p_heavy, and the
// heavy row's side B^T p_row summed over the 64 lanes by a fixed butterfly into part[0..OD).  B is
// 3 x OD in the row's orientation, stored per lane as 3-column sub-blocks (row-major 3 x 3 + one pad
// = five double2 each; OD = 1: three values in two double2), taken one sub-block at a time so
// the live registers stay those of a 3 x 3 slot.
// columns [0, nc) of a 3 x 3 sub-block B (row-major, row stride 3; nc <= 3, the rest zero)
__device__ __forceinline__ void heavy_cols(const double *B, int nc, int64_t oh, const double *__restrict__ zp,
                                           double beta, const double pv[3], double acc[6], double *__restrict__ part,
                                           int lane) {
    double ph[3], cc[3];
#pragma unroll
    for (int j = 0; j < 3; j++) ph[j] = j < nc ? pval(zp, beta, oh + j) : 0.0;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) acc[i] += B[i * 3 + j] * ph[j];
#pragma unroll
    for (int j = 0; j < 3; j++) cc[j] = (B[j] * pv[0] + B[3 + j] * pv[1]) + B[6 + j] * pv[2];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
        for (int j = 0; j < 3; j++) cc[j] += __shfl_xor(cc[j], off, 64);
    if (lane < nc) part[lane] = lane == 0 ? cc[0] : lane == 1 ? cc[1] : cc[2];
}

__device__ __forceinline__ void heavy_slot(const double2 *__restrict__ hb, int od, int64_t oh,
                                           const double *__restrict__ zp, double beta, const double pv[3], double acc[6],
                                           double *__restrict__ part, int lane) {
    if (od == 1) {
        const double2 t0 = hb[0], t1 = hb[64];
        const double B[9] = {t0.x, 0.0, 0.0, t0.y, 0.0, 0.0, t1.x, 0.0, 0.0};
        heavy_cols(B, 1, oh, zp, beta, pv, acc, part, lane);
        return;
    }
    for (int sb = 0; 3 * sb < od; sb++) {
        double B[10];
#pragma unroll
        for (int q2 = 0; q2 < 5; q2++) {
            const double2 t = hb[(5 * sb + q2) * 64];
            B[2 * q2] = t.x;
            B[2 * q2 + 1] = t.y;
        }
        heavy_cols(B, min(3, od - 3 * sb), oh + 3 * sb, zp, beta, pv, acc, part + 3 * sb, lane);
    }
}

// sliced rows' 3x3 blocks -> slot-major, lane-interleaved copies in the rows' orientation
__global__ void __launch_bounds__(256) k_pcg_repack(const PcgDev G, const double *__restrict__ hval) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= G.nslots * 64) {
        // heavy slots: 3 x od blocks (row orientation) into 3 x 6, zero padded
        const int64_t u = t - G.nslots * 64;
        if (u >= G.nhslots * 64) return;
        const int64_t g = u >> 6;
        const int64_t m = G.hs_map[u];
        double2 *dst = reinterpret_cast<double2 *>(G.hs_val) + G.hs_voff[g] + (u & 63);
        const int od = G.vdim[G.heavy_v[G.hs_hk[g]]];
        const double *h = hval + (m < 0 ? 0 : (m & ((1LL << 62) - 1)));
        const bool tr = m >= 0 && ((m >> 62) & 1);
        double B[18];                          // B[i][j] of the 3 x od block, row orientation
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 6; j++) B[i * 6 + j] = (m >= 0 && j < od) ? (tr ? h[j * 3 + i] : h[i * od + j]) : 0.0;
        if (od == 1) {
            dst[0] = make_double2(B[0], B[6]);
            dst[64] = make_double2(B[12], 0.0);
            return;
        }
#pragma unroll
        for (int sb = 0; sb < 2; sb++) {
            if (3 * sb >= od) break;
            double v[10];
#pragma unroll
            for (int i = 0; i < 3; i++)
#pragma unroll
                for (int j = 0; j < 3; j++) v[i * 3 + j] = B[i * 6 + 3 * sb + j];
            v[9] = 0.0;
#pragma unroll
            for (int q2 = 0; q2 < 5; q2++) dst[(5 * sb + q2) * 64] = make_double2(v[2 * q2], v[2 * q2 + 1]);
        }
        return;
    }
    const int64_t m = G.sl_map[t];
    double2 *dst = reinterpret_cast<double2 *>(G.sl_val) + (t >> 6) * 320 + (t & 63);
    double v[10];
    if (m < 0) {
#pragma unroll
        for (int q = 0; q < 9; q++) v[q] = 0.0;
    } else {
        const double *h = hval + (m & ((1LL << 62) - 1));
        const bool tr = (m >> 62) & 1;
        double u[9];
#pragma unroll
        for (int q = 0; q < 9; q++) u[q] = h[q];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) v[i * 3 + j] = tr ? u[j * 3 + i] : u[i * 3 + j];
    }
    v[9] = __longlong_as_double((long long)G.sl_col[t]);
#pragma unroll
    for (int q2 = 0; q2 < 5; q2++) dst[q2 * 64] = make_double2(v[2 * q2], v[2 * q2 + 1]);
}

// per vertex: M_v = (H_vv + lambda I)^-1 through its Cholesky factor; r = b, z = M r, x = 0, p = 0
__global__ void __launch_bounds__(256) k_pcg_setup(const PcgDev G, const double *__restrict__ hval,
                                                   const double *__restrict__ b, double lam, double *__restrict__ x) {
    __shared__ double red[2][256];
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    double rz = 0.0, rr = 0.0;
    if (v < G.nv) {
        const int d = G.vdim[v];
        const int64_t o = G.voff[v];
        const double *D = G.mf ? G.mf_diag + G.moff[v] : hval + G.diag_off[v];
        double A[36];
#pragma unroll
        for (int i = 0; i < 6; i++)
#pragma unroll
            for (int j = 0; j < 6; j++) A[i * 6 + j] = (i < d && j < d) ? D[i * d + j] + (i == j ? lam : 0.0) : 0.0;
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 6; j++) {
            if (j < d) {
                double s = A[j * 6 + j];
#pragma unroll
                for (int k = 0; k < j; k++) s -= A[j * 6 + k] * A[j * 6 + k];
                if (!(s > 0.0)) ok = false;
                s = sqrt(s);
                A[j * 6 + j] = s;
#pragma unroll
                for (int i = j + 1; i < 6; i++) {
                    if (i < d) {
                        double t = A[i * 6 + j];
#pragma unroll
                        for (int k = 0; k < j; k++) t -= A[i * 6 + k] * A[j * 6 + k];
                        A[i * 6 + j] = t / s;
                    }
                }
            }
        }
        if (!ok) G.rec[PR_STATUS] = kPcgBadBlock;   // record 0 (cleared before the launch)
        double *M = G.minv + G.moff[v];
        // z = M r accumulated column by column as M's columns are formed: z_i += M_ic r_c in c order,
        // the same FMA sequence as a row-wise sum after the fact, without holding all of M (VGPRs)
        double rv[6], z[6];
#pragma unroll
        for (int i = 0; i < 6; i++) { rv[i] = i < d ? b[o + i] : 0.0; z[i] = 0.0; }
#pragma unroll
        for (int c = 0; c < 6; c++) {
            if (c < d) {
                double y[6];
#pragma unroll
                for (int i = 0; i < 6; i++) {
                    double t = (i == c) ? 1.0 : 0.0;
#pragma unroll
                    for (int k = 0; k < i; k++) t -= A[i * 6 + k] * y[k];
                    y[i] = (i < d) ? t / A[i * 6 + i] : 0.0;
                }
#pragma unroll
                for (int i = 5; i >= 0; i--) {
                    if (i < d) {
                        double t = y[i];
#pragma unroll
                        for (int k = i + 1; k < 6; k++)
                            if (k < d) t -= A[k * 6 + i] * y[k];
                        y[i] = t / A[i * 6 + i];
                    }
                }
#pragma unroll
                for (int i = 0; i < 6; i++)
                    if (i < d) { M[i * d + c] = y[i]; z[i] += y[i] * rv[c]; }
            }
        }
        double2 *zp = reinterpret_cast<double2 *>(G.zp);
#pragma unroll
        for (int i = 0; i < 6; i++) {
            if (i < d) {
                const double zi = z[i];
                G.r[o + i] = rv[i];
                zp[o + i] = make_double2(zi, 0.0);
                x[o + i] = 0.0;
                rz += rv[i] * zi;
                rr += rv[i] * rv[i];
            }
        }
    }
    wg_pair_tree(rz, rr, red, G.partB + 2 * blockIdx.x);
}

// the sliced rows (one workgroup per slice); the heavy rows and the generic light rows follow in
// k_pcg_heavy (their own launch: this kernel's register budget is the slices')
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DEFTRI_PCG_WPE))) k_pcg_product(int it, const PcgDev G, const double *__restrict__ hval,
                                                     double lam) {
    __shared__ double red[6][256];
    double *rec = G.rec + kPcgRec * (it + 1);
    const double *prv = G.rec + kPcgRec * it;
    const int tid = threadIdx.x;
    if (prv[PR_STATUS] != 0.0) {                     // converged / failed earlier: carry the verdict
        if (blockIdx.x == 0 && tid == 0) { rec[PR_STATUS] = prv[PR_STATUS]; rec[PR_ITS] = prv[PR_ITS]; }
        return;
    }
    double rz, rr;
    wg_sum2(G.partB, G.nB, rz, rr, red);
    const double bb = it == 0 ? rr : G.rec[kPcgRec + PR_RR];
    const bool conv = rr <= G.tol2 * bb;
    if (blockIdx.x == 0 && tid == 0) {
        rec[PR_RZ] = rz;
        rec[PR_RR] = rr;
        rec[PR_STATUS] = conv ? kPcgConverged : kPcgRunning;
        rec[PR_ITS] = it;
    }
    if (conv) return;
    const double beta = it == 0 ? 0.0 : rz / prv[PR_RZ];
    const double *zp = G.zp;
    double2 *pq2 = reinterpret_cast<double2 *>(G.pq);
    {
        // sliced rows: one slice (64 rows, lane = row) per workgroup; its four waves take every
        // fourth slot of each kind, so a wave's dependent chain (column index -> gather) is a
        // quarter of the slice's; every load is coalesced but the (z, p_prev) gathers.  The four
        // partial row sums meet in LDS in a fixed order.
        const int sl = blockIdx.x;
        const bool live = sl < G.nsl;              // the launch has one workgroup even with no slices
        const int w = tid >> 6, lane = tid & 63;
        const int v = live ? G.sl_v[sl * 64 + lane] : -1;
        const int64_t o = v >= 0 ? G.voff[v] : 0;
        double pv[3];
#pragma unroll
        for (int i = 0; i < 3; i++) pv[i] = v >= 0 ? pval(zp, beta, o + i) : 0.0;
        double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        const int64_t g0 = live ? G.sl_off[sl] : 0;
        const int ns = live ? G.sl_n[sl] : 0;
        constexpr int kSlotBatch = DEFTRI_PCG_BATCH;   // slots of one wave in flight together
        const double2 *slv = reinterpret_cast<const double2 *>(G.sl_val);
        for (int k0 = w; k0 < ns; k0 += 4 * kSlotBatch) {
            // per lane and slot: five 16-byte loads = the 3x3 block + the column dof
            int c[kSlotBatch];
            double h[kSlotBatch][10], pj[kSlotBatch][3];
#pragma unroll
            for (int u = 0; u < kSlotBatch; u++) {
                const bool in = k0 + 4 * u < ns;
                const double2 *hv = slv + (g0 + k0 + 4 * u) * 320 + lane;
#pragma unroll
                for (int q2 = 0; q2 < 5; q2++) {
                    const double2 t = in ? hv[q2 * 64] : make_double2(0.0, 0.0);
                    h[u][2 * q2] = t.x;
                    h[u][2 * q2 + 1] = t.y;
                }
                c[u] = in ? (int)__double_as_longlong(h[u][9]) : -1;
            }
#pragma unroll
            for (int u = 0; u < kSlotBatch; u++)
#pragma unroll
                for (int j = 0; j < 3; j++) pj[u][j] = c[u] >= 0 ? pval(zp, beta, c[u] + j) : 0.0;
#pragma unroll
            for (int u = 0; u < kSlotBatch; u++)
                if (c[u] >= 0)
#pragma unroll
                    for (int i = 0; i < 3; i++)
#pragma unroll
                        for (int j = 0; j < 3; j++) acc[i] += h[u][i * 3 + j] * pj[u][j];
        }
        // couplings to heavy vertices: the row side B p_heavy, and the heavy row's side B^T p_row
        // reduced over the slice's lanes (fixed butterfly) into the slot's partial
        const int64_t h0 = live ? G.sl_hoff[sl] : 0;
        const int nh = live ? G.sl_hn[sl] : 0;
        for (int k = w; k < nh; k += 4) {
            const int64_t g = h0 + k;
            const int hv = G.heavy_v[G.hs_hk[g]];
            const int64_t oh = G.voff[hv];
            const double2 *hb = reinterpret_cast<const double2 *>(G.hs_val) + G.hs_voff[g] + lane;
            double *part = G.hs_part + G.hs_pos[g] * 6;     // heavy-vertex-major: k_pcg_heavy reads runs
            heavy_slot(hb, G.vdim[hv], oh, zp, beta, pv, acc, part, lane);
        }
        const int64_t x0 = live ? G.sl_xoff[sl] : 0;
        const int nx = live ? G.sl_nx[sl] : 0;
        for (int k = w; k < nx; k += 4) {
            const PcgEnt E = load_ent(G.sl_x, (x0 + k) * 64 + lane);
            if (E.odim) ent_acc(E, 3, hval, zp, beta, acc);
        }
#pragma unroll
        for (int i = 0; i < 3; i++) red[i][tid] = acc[i];
        __syncthreads();
        double pqs = 0.0;
        if (w == 0 && v >= 0) {
#pragma unroll
            for (int i = 0; i < 3; i++) {
                const double a = (red[i][lane] + red[i][64 + lane]) + (red[i][128 + lane] + red[i][192 + lane]);
                const double qv = a + lam * pv[i];
                pq2[o + i] = make_double2(pv[i], qv);
                pqs += pv[i] * qv;
            }
        }
        __syncthreads();
        const double s = wg_tree(pqs, red[3]);
        if (tid == 0 && sl < G.nsl) G.partA[blockIdx.x] = s;
        return;
    }
}

// After the sliced product, iteration it: one workgroup per heavy dof — q = (its slots' partials,
// fixed tree) + (the heavy row's remaining entries: its diagonal block and couplings outside the
// slices, fixed tree) + lambda p — then the generic light rows, one thread each (their p.q partials
// follow the slices' in partA).  beta comes from the record the product's workgroup 0 wrote.
__global__ void __launch_bounds__(256) k_pcg_heavy(int it, const PcgDev G, const double *__restrict__ hval,
                                                   double lam) {
    __shared__ double red[256];
    const double *rec = G.rec + kPcgRec * (it + 1);
    const double *zp = G.zp;
    double2 *pq2 = reinterpret_cast<double2 *>(G.pq);
    const int tid = threadIdx.x;
    // the partial sums below need no scalar of this iteration: they are loaded and summed before the
    // status test (uniform per workgroup), beta only after it
    if (G.mf && (int)blockIdx.x == G.nheavy_dofs) {
        // matrix-free plans (no light rows): the product's p.q partials, once, in a fixed order
        const int nA = G.nA_sl;
        const double a = wg_tree([&] {
            double t = 0.0;
            for (int i = tid; i < nA; i += 256) t += G.partA[i];
            return t;
        }(), red);
        if (rec[PR_STATUS] != 0.0) return;
        if (tid == 0) G.rec[kPcgRec * (it + 1) + PR_PQA] = a;
        return;
    }
    if ((int)blockIdx.x >= G.nheavy_dofs) {
        if (rec[PR_STATUS] != 0.0) return;
        const double beta = it == 0 ? 0.0 : rec[PR_RZ] / G.rec[kPcgRec * it + PR_RZ];
        const int k = (blockIdx.x - G.nheavy_dofs) * 256 + tid;
        double pqs = 0.0;
        if (k < G.nlight) {
            const int v = G.light_v[k];
            const int d = G.vdim[v];
            const int64_t o = G.voff[v];
            double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
            const int64_t e1 = G.ent_begin[v + 1];
            for (int64_t e = G.ent_begin[v]; e < e1; e++) ent_acc(load_ent(G.ent, e), d, hval, zp, beta, acc);
#pragma unroll
            for (int i = 0; i < 6; i++) {
                if (i < d) {
                    const double pv = pval(zp, beta, o + i);
                    const double qv = acc[i] + lam * pv;
                    pq2[o + i] = make_double2(pv, qv);
                    pqs += pv * qv;
                }
            }
        }
        const double s = wg_tree(pqs, red);
        if (tid == 0) G.partA[G.nA_sl + blockIdx.x - G.nheavy_dofs] = s;
        return;
    }
    const int k = blockIdx.x;
    int hk = 0;
    while (G.h_dofbase[hk + 1] <= k) hk++;
    const int i = k - G.h_dofbase[hk];
    const int64_t b0 = G.hv_slot_begin[hk], b1 = G.hv_slot_begin[hk + 1];
    // four independent strided streams per thread, combined in order; four rounds of the streams
    // (16 loads) are issued before any is added, so a heavy dof of up to 4096 slots waits on one
    // round of load latency (same additions in the same order as a round-by-round loop)
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    for (int64_t t0 = b0 + tid; t0 < b1; t0 += 4096) {
        double h[16];
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int64_t t = t0 + 256 * q;
            h[q] = t < b1 ? G.hs_part[t * 6 + i] : 0.0;
        }
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (t0 + 1024 * r + 256 * u < b1) a[u] += h[4 * r + u];
    }
    const double s_slots = wg_tree((a[0] + a[1]) + (a[2] + a[3]), red);
    if (rec[PR_STATUS] != 0.0) return;
    const double beta = it == 0 ? 0.0 : rec[PR_RZ] / G.rec[kPcgRec * it + PR_RZ];
    const int v = G.heavy_v[hk];
    const int d = G.vdim[v];
    const int f0 = G.h_first[hk], f1 = G.h_first[hk + 1];
    const int64_t e0 = f0 < f1 ? G.hc_beg[f0] : 0, e1 = f0 < f1 ? G.hc_end[f1 - 1] : 0;
    double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int64_t e = e0 + tid; e < e1; e += 256) ent_acc(load_ent(G.hres, e), d, hval, zp, beta, acc);
    double ai = acc[0];
#pragma unroll
    for (int u = 1; u < 6; u++) ai = i == u ? acc[u] : ai;
    const double s_rest = wg_tree(ai, red);
    if (tid == 0) {
        const int64_t o = G.voff[v] + i;
        const double pv = pval(zp, beta, o);
        pq2[o] = make_double2(pv, 0.0);
        G.hqf[k] = (s_slots + s_rest) + lam * pv;
    }
}

__global__ void __launch_bounds__(256) k_pcg_update(int it, const PcgDev G, double lam, double *__restrict__ x) {
    __shared__ double red[2][256];
    double *rec = G.rec + kPcgRec * (it + 1);
    const int tid = threadIdx.x;
    const double2 *pq2 = reinterpret_cast<const double2 *>(G.pq);
    // a 3-dof row (a point, not a heavy row) loads everything it needs that does not depend on alpha
    // first — (p, q), r, x and M — so those loads are in flight while the status, the p.q sums and
    // the heavy rows arrive; the arithmetic below is the generic path's, in the same order
    const int64_t v = (int64_t)blockIdx.x * 256 + tid;
    int d = 0, hk = -1;
    int64_t o = 0;
    bool fast = false;
    double2 w3[3];
    double r3[3], x3[3], M9[9];
    if (v < G.nv) {
        d = G.vdim[v];
        o = G.voff[v];
        hk = G.v_heavy[v];
        fast = d == 3 && hk < 0;
        if (fast) {
            const double *M = G.minv + G.moff[v];
#pragma unroll
            for (int i = 0; i < 3; i++) { w3[i] = pq2[o + i]; r3[i] = G.r[o + i]; x3[i] = x[o + i]; }
#pragma unroll
            for (int k = 0; k < 9; k++) M9[k] = M[k];
        }
    }
    if (rec[PR_STATUS] != 0.0) return;
    const int nA = G.nA_sl + G.nA_light;
    const double pq_light = G.mf ? rec[PR_PQA] : wg_tree([&] {
        double a = 0.0;
        for (int i = tid; i < nA; i += 256) a += G.partA[i];
        return a;
    }(), red[0]);
    // the heavy rows' p.q (their q from k_pcg_heavy), in heavy-dof order
    if (tid == 0) {
        double a = 0.0;
        for (int hh = 0; hh < G.nheavy; hh++) {
            const int64_t oh = G.voff[G.heavy_v[hh]];
            for (int i = 0; i < G.h_dofbase[hh + 1] - G.h_dofbase[hh]; i++) a += pq2[oh + i].x * G.hqf[G.h_dofbase[hh] + i];
        }
        red[1][0] = a;
    }
    __syncthreads();
    const double pq = pq_light + red[1][0];
    const double alpha = rec[PR_RZ] / pq;
    if (!(pq > 0.0) || !isfinite(alpha)) {
        if (blockIdx.x == 0 && tid == 0) rec[PR_STATUS] = kPcgBreakdown;
        return;
    }
    if (blockIdx.x == 0 && tid == 0) { rec[PR_PQ] = pq; rec[PR_ALPHA] = alpha; }
    __syncthreads();
    double rz = 0.0, rr = 0.0;
    if (fast) {
        double rv[3];
        double2 *zp = reinterpret_cast<double2 *>(G.zp);
#pragma unroll
        for (int i = 0; i < 3; i++) {
            x[o + i] = x3[i] + alpha * w3[i].x;
            rv[i] = r3[i] - alpha * w3[i].y;
            G.r[o + i] = rv[i];
        }
#pragma unroll
        for (int i = 0; i < 3; i++) {
            double zi = 0.0;
#pragma unroll
            for (int j = 0; j < 3; j++) zi += M9[i * 3 + j] * rv[j];
            zp[o + i] = make_double2(zi, w3[i].x);
            rz += rv[i] * zi;
            rr += rv[i] * rv[i];
        }
    } else if (v < G.nv) {
        double rv[6], pv[6];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            rv[i] = 0.0;
            pv[i] = 0.0;
            if (i < d) {
                const double2 w = pq2[o + i];
                const double qv = hk < 0 ? w.y : G.hqf[G.h_dofbase[hk] + i];
                pv[i] = w.x;
                x[o + i] += alpha * w.x;
                rv[i] = G.r[o + i] - alpha * qv;
                G.r[o + i] = rv[i];
            }
        }
        const double *M = G.minv + G.moff[v];
        double2 *zp = reinterpret_cast<double2 *>(G.zp);
#pragma unroll
        for (int i = 0; i < 6; i++) {
            if (i < d) {
                double zi = 0.0;
#pragma unroll
                for (int j = 0; j < 6; j++)
                    if (j < d) zi += M[i * d + j] * rv[j];
                zp[o + i] = make_double2(zi, pv[i]);
                rz += rv[i] * zi;
                rr += rv[i] * rv[i];
            }
        }
    }
    wg_pair_tree(rz, rr, red, G.partB + 2 * blockIdx.x);
}


// ---- matrix-free product (pcg.h) ----------------------------------------------------------------
__device__ __forceinline__ void mf_rec(int64_t r, int &kind, int &mask, int &hs, int &base, int64_t &e) {
    kind = (int)((uint64_t)r >> 62);
    mask = (int)((r >> 58) & 0xf);
    hs = (int)((r >> 55) & 0x7);
    base = (int)((r >> 40) & 0x7fff);
    e = r & 0xffffffffffLL;
}

// fixed butterfly over the wave, then the four waves in order: one value per call
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

#ifndef DEFTRI_MF_WPE
#define DEFTRI_MF_WPE 4
#endif
// matrix-free plans, before product it: the update's (r.z, r.r) partials summed once (fixed order),
// the convergence test and the record of iteration it (carried over when an earlier one ended)
__global__ void __launch_bounds__(256) k_pcg_dots(int it, const PcgDev G) {
    __shared__ double red[2][256];
    double *rec = G.rec + kPcgRec * (it + 1);
    const double *prv = G.rec + kPcgRec * it;
    if (prv[PR_STATUS] != 0.0) {
        if (threadIdx.x == 0) { rec[PR_STATUS] = prv[PR_STATUS]; rec[PR_ITS] = prv[PR_ITS]; }
        return;
    }
    double rz, rr;
    wg_sum2(G.partB, G.nB, rz, rr, red);
    if (threadIdx.x == 0) {
        const double bb = it == 0 ? rr : G.rec[kPcgRec + PR_RR];
        rec[PR_RZ] = rz;
        rec[PR_RR] = rr;
        rec[PR_STATUS] = rr <= G.tol2 * bb ? kPcgConverged : kPcgRunning;
        rec[PR_ITS] = it;
    }
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DEFTRI_MF_WPE))) k_mf_product(int it, const PcgDev G, double lam) {
    extern __shared__ double C[];                     // per local edge and in-slice role: J^T s
    __shared__ double red[4][256];
    double *rec = G.rec + kPcgRec * (it + 1);
    const double *prv = G.rec + kPcgRec * it;
    const int tid = threadIdx.x;
    const int sl = blockIdx.x;
    const bool live = sl < G.nsl;
    const int w = tid >> 6, lane = tid & 63;
    // The workgroup's chain of dependent loads bounds this kernel (SQ: ~70 % of wave cycles
    // waiting), so every load that does not need this iteration's scalars is issued first and stays
    // in flight while the status and the (r.z, r.r) partials arrive: the slice's metadata (one
    // 32-byte record), then the row, its first local edge, its first incidence slots, its first own
    // edge, then their dofs / Jacobians / weights.
    int64_t l0 = 0, i0 = 0, o0 = 0;
    int ne = 0, ni = 0, no = 0, nt = 0, nh = 0;
    if (live) {
        const longlong2 m0 = reinterpret_cast<const longlong2 *>(G.mf_sl_meta)[2 * sl];
        const longlong2 m1 = reinterpret_cast<const longlong2 *>(G.mf_sl_meta)[2 * sl + 1];
        l0 = m0.x; i0 = m0.y; o0 = m1.x;
        const int64_t c = m1.y;
        ne = (int)(c & 0xffff); ni = (int)((c >> 16) & 0xff); no = (int)((c >> 24) & 0xff);
        nt = (int)((c >> 32) & 0xf); nh = (int)((c >> 36) & 0xf);
    }
    const int v = live ? G.sl_v[sl * 64 + lane] : -1;
    // first local edge of this thread
    const bool has1 = tid < ne;
    int kind1 = 0, mask1 = 0, hs1 = 0, base1 = 0;
    int64_t e1 = 0;
    if (has1) mf_rec(G.mf_le[l0 + tid], kind1, mask1, hs1, base1, e1);
    // incidence slots (every fourth, the first kPre) and the first own edge of this wave
    constexpr int kPre = 4;
    int offs[kPre];
#pragma unroll
    for (int u = 0; u < kPre; u++) offs[u] = (w + 4 * u < ni) ? G.mf_inc[(i0 + w + 4 * u) * 64 + lane] : -1;
    const int x1 = w < no ? G.mf_own[(o0 + w) * 64 + lane] : -1;
    int4 d1 = make_int4(0, 0, 0, 0);
    int td1 = 0;
    double J1[18], W1 = 0.0;
#pragma unroll
    for (int q = 0; q < 18; q++) J1[q] = 0.0;
    if (has1) {
        d1 = reinterpret_cast<const int4 *>(G.mf_adof)[e1];
        td1 = G.mf_atdof[e1];
        const double2 *J2 = reinterpret_cast<const double2 *>(G.Jarap) + 9 * e1;
#pragma unroll
        for (int q = 0; q < 9; q++) { const double2 t = J2[q]; J1[2 * q] = t.x; J1[2 * q + 1] = t.y; }
        W1 = G.Warap[e1];
    }
    // the own edge: reprojection J (2 x 3) + W, or depth J (4) + W + the scale's dof
    double Jo[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, Wo = 0.0;
    int so = 0;
    if (x1 >= 0) {
        const int64_t e = x1 & ((1 << 27) - 1);
        if (!(x1 >> 30)) {
            const double2 *J2 = reinterpret_cast<const double2 *>(G.Jrep) + 3 * e;
#pragma unroll
            for (int q = 0; q < 3; q++) { const double2 t = J2[q]; Jo[2 * q] = t.x; Jo[2 * q + 1] = t.y; }
            Wo = G.Wrep[e];
        } else {
            const double2 *J2 = reinterpret_cast<const double2 *>(G.Jdep) + 2 * e;
#pragma unroll
            for (int q = 0; q < 2; q++) { const double2 t = J2[q]; Jo[2 * q] = t.x; Jo[2 * q + 1] = t.y; }
            Wo = G.Wdep[e];
            so = G.mf_ddof[2 * e + 1];
        }
    }
    const int64_t o = v >= 0 ? G.voff[v] : 0;
    if (rec[PR_STATUS] != 0.0) return;                // k_pcg_dots: converged / failed
    const double beta = it == 0 ? 0.0 : rec[PR_RZ] / prv[PR_RZ];
    const double *zp = G.zp;
    double pv[3];
#pragma unroll
    for (int i = 0; i < 3; i++) pv[i] = v >= 0 ? pval(zp, beta, o + i) : 0.0;
    // phase A: s_e = W_e (J_e p) per local (ARAP) edge, J_{e,v}^T s_e into LDS for the in-slice
    // roles, the owned edges' T_g parts
    double hT[kMfMaxT][6];
#pragma unroll
    for (int h = 0; h < kMfMaxT; h++)
#pragma unroll
        for (int i = 0; i < 6; i++) hT[h][i] = 0.0;
    for (int k = tid; k < ne; k += 256) {
        if (k != tid) {                               // later passes load here (the first is prefetched)
            mf_rec(G.mf_le[l0 + k], kind1, mask1, hs1, base1, e1);
            d1 = reinterpret_cast<const int4 *>(G.mf_adof)[e1];
            td1 = G.mf_atdof[e1];
            const double2 *J2 = reinterpret_cast<const double2 *>(G.Jarap) + 9 * e1;
#pragma unroll
            for (int q = 0; q < 9; q++) { const double2 t = J2[q]; J1[2 * q] = t.x; J1[2 * q + 1] = t.y; }
            W1 = G.Warap[e1];
        }
        double dot = 0.0;
#pragma unroll
        for (int i = 0; i < 3; i++) dot += J1[i] * pval(zp, beta, d1.x + i);
#pragma unroll
        for (int i = 0; i < 3; i++) dot += J1[3 + i] * pval(zp, beta, d1.y + i);
#pragma unroll
        for (int i = 0; i < 3; i++) dot += J1[6 + i] * pval(zp, beta, d1.z + i);
#pragma unroll
        for (int i = 0; i < 3; i++) dot += J1[9 + i] * pval(zp, beta, d1.w + i);
#pragma unroll
        for (int i = 0; i < 6; i++) dot += J1[12 + i] * pval(zp, beta, td1 + i);
        const double sv = W1 * dot;
        int pos = base1;                              // the roles whose point is in this slice
#pragma unroll
        for (int r = 0; r < 4; r++)
            if ((mask1 >> r) & 1) {
#pragma unroll
                for (int i = 0; i < 3; i++) C[pos + i] = J1[3 * r + i] * sv;
                pos += 3;
            }
        if (hs1 > 0)
#pragma unroll
            for (int h = 0; h < kMfMaxT; h++)
                if (h == hs1 - 1)
#pragma unroll
                    for (int i = 0; i < 6; i++) hT[h][i] += J1[12 + i] * sv;
    }
    // the owned edges' T_g partials: per slot, butterfly per wave, waves in order
    for (int h = 0; h < nt; h++) {
        double hh[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int q = 0; q < kMfMaxT; q++)
            if (q == h)
#pragma unroll
                for (int i = 0; i < 6; i++) hh[i] = hT[q][i];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            const double x = wave_sum(hh[i]);
            if (lane == 0) red[0][4 * i + w] = x;     // 6 values x 4 waves
        }
        __syncthreads();
        if (tid < 6) {
            const double *r4 = &red[0][4 * tid];
            G.hs_part[(int64_t)G.mf_sl_hpos[sl * kMfMaxH + h] * 6 + tid] = (r4[0] + r4[1]) + (r4[2] + r4[3]);
        }
        __syncthreads();
    }
    __syncthreads();
    // phase B: lane = row; the four waves take every fourth incidence slot and every fourth own
    // (single-point) edge slot; partial rows meet in LDS in a fixed order
    double acc[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int u = 0; u < kPre; u++)
        if (offs[u] >= 0)
#pragma unroll
            for (int i = 0; i < 3; i++) acc[i] += C[offs[u] + i];
    for (int k = w + 4 * kPre; k < ni; k += 4) {
        const int off = G.mf_inc[(i0 + k) * 64 + lane];
        if (off >= 0)
#pragma unroll
            for (int i = 0; i < 3; i++) acc[i] += C[off + i];
    }
    double hS[kMfMaxS] = {0.0, 0.0, 0.0, 0.0};
    auto own_edge = [&](int x, const double (&J)[6], double wv, int sd) __attribute__((always_inline)) {
        const int ss = (x >> 27) & 7;
        if (!(x >> 30)) {                              // reprojection (2 rows)
            const double s0 = wv * ((J[0] * pv[0] + J[1] * pv[1]) + J[2] * pv[2]);
            const double s1 = wv * ((J[3] * pv[0] + J[4] * pv[1]) + J[5] * pv[2]);
#pragma unroll
            for (int i = 0; i < 3; i++) acc[i] += J[i] * s0 + J[3 + i] * s1;
        } else {                                       // depth (point, scale)
            const double sv = wv * (((J[0] * pv[0] + J[1] * pv[1]) + J[2] * pv[2]) + J[3] * pval(zp, beta, sd));
#pragma unroll
            for (int i = 0; i < 3; i++) acc[i] += J[i] * sv;
#pragma unroll
            for (int q = 0; q < kMfMaxS; q++)
                if (q == ss - 1) hS[q] += J[3] * sv;
        }
    };
    if (x1 >= 0) own_edge(x1, Jo, Wo, so);
    for (int k = w + 4; k < no; k += 4) {
        const int x = G.mf_own[(o0 + k) * 64 + lane];
        if (x < 0) continue;
        const int64_t e = x & ((1 << 27) - 1);
        double J[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        double wv;
        int sd = 0;
        if (!(x >> 30)) {
#pragma unroll
            for (int q = 0; q < 6; q++) J[q] = G.Jrep[6 * e + q];
            wv = G.Wrep[e];
        } else {
#pragma unroll
            for (int q = 0; q < 4; q++) J[q] = G.Jdep[4 * e + q];
            wv = G.Wdep[e];
            sd = G.mf_ddof[2 * e + 1];
        }
        own_edge(x, J, wv, sd);
    }
    // the scale partials: per slot, butterfly per wave, waves in order
    for (int j = 0; j < nh - nt; j++) {
        double hh = 0.0;
#pragma unroll
        for (int q = 0; q < kMfMaxS; q++)
            if (q == j) hh = hS[q];
        const double x = wave_sum(hh);
        if (lane == 0) red[3][w] = x;
        __syncthreads();
        if (tid == 0)
            G.hs_part[(int64_t)G.mf_sl_hpos[sl * kMfMaxH + nt + j] * 6] = (red[3][0] + red[3][1]) + (red[3][2] + red[3][3]);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 3; i++) red[i][tid] = acc[i];
    __syncthreads();
    double pqs = 0.0;
    double2 *pq2 = reinterpret_cast<double2 *>(G.pq);
    if (w == 0 && v >= 0) {
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const double a = (red[i][lane] + red[i][64 + lane]) + (red[i][128 + lane] + red[i][192 + lane]);
            const double qv = a + lam * pv[i];
            pq2[o + i] = make_double2(pv[i], qv);
            pqs += pv[i] * qv;
        }
    }
    // p.q of the slice: only wave 0 holds rows, so one fixed butterfly (no workgroup barrier)
    if (w == 0) {
        const double sum = wave_sum(pqs);
        if (lane == 0 && live) G.partA[blockIdx.x] = sum;
    }
}

// lower-triangle index of (a, b), a >= b, in a 6 x 6 block
__device__ __forceinline__ int tri6(int a, int b) { return a * (a + 1) / 2 + b; }

// per LM iteration: point rows' diagonal blocks and b from their incidences; the owned edges' heavy
// diagonal blocks and b as per-slot partials (k_mf_lin_heavy sums them)
__global__ void __launch_bounds__(256) k_mf_lin(const PcgDev G) {
    __shared__ double red[12][256];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int sl = blockIdx.x;
    const int64_t l0 = G.mf_le_off[sl];
    const int ne = G.mf_le_n[sl];
    const int nh = G.sl_hn[sl], nt = G.mf_sl_nt[sl];
    // T_g slots: the owned ARAP edges' 6 x 6 blocks (lower triangle) and b parts
    for (int h = 0; h < nt; h++) {
        double a[kMfLin];
#pragma unroll
        for (int q = 0; q < kMfLin; q++) a[q] = 0.0;
        for (int k = tid; k < ne; k += 256) {
            int kind, mask, hs, base;
            int64_t e;
            mf_rec(G.mf_le[l0 + k], kind, mask, hs, base, e);
            if (hs != h + 1) continue;
            const double *J = G.Jarap + 18 * e + 12;
            const double wv = G.Warap[e], er = G.Earap[e];
#pragma unroll
            for (int i = 0; i < 6; i++) {
                const double ai = J[i] * wv;
#pragma unroll
                for (int j = 0; j <= i; j++) a[tri6(i, j)] += ai * J[j];
                a[21 + i] -= J[i] * (wv * er);
            }
        }
        double *out = G.mf_hlin + G.hs_pos[G.sl_hoff[sl] + h] * kMfLin;
        for (int q0 = 0; q0 < kMfLin; q0 += 12) {
#pragma unroll
            for (int q = 0; q < 12; q++) {
                double vq = 0.0;
#pragma unroll
                for (int u = 0; u < kMfLin; u++)
                    if (u == q0 + q) vq = a[u];
                vq = wave_sum(vq);
                if (lane == 0) red[q][w] = vq;
            }
            __syncthreads();
            if (tid < 12 && q0 + tid < kMfLin)
                out[q0 + tid] = (red[tid][0] + red[tid][1]) + (red[tid][2] + red[tid][3]);
            __syncthreads();
        }
    }
    // point rows: their ARAP incidences, then their own reprojection / depth edges
    const int v = G.sl_v[sl * 64 + lane];
    double acc[12];
#pragma unroll
    for (int q = 0; q < 12; q++) acc[q] = 0.0;
    auto add_rows = [&](const double *J, int m, double wv, double er0, double er1) {
        for (int r = 0; r < m; r++) {
            const double er = r == 0 ? er0 : er1;
#pragma unroll
            for (int i = 0; i < 3; i++) {
                const double ai = J[3 * r + i] * wv;
#pragma unroll
                for (int j = 0; j < 3; j++) acc[3 * i + j] += ai * J[3 * r + j];
                acc[9 + i] -= J[3 * r + i] * (wv * er);
            }
        }
    };
    const int64_t i0 = G.mf_in_off[sl];
    const int ni = G.mf_in_n[sl];
    for (int k = w; k < ni; k += 4) {
        const int ir = G.mf_inc2[(i0 + k) * 64 + lane];
        if (ir < 0) continue;
        const int kl = ir >> 2, role = ir & 3;
        int kind, mask, hs, base;
        int64_t e;
        mf_rec(G.mf_le[l0 + kl], kind, mask, hs, base, e);
        add_rows(G.Jarap + 18 * e + 3 * role, 1, G.Warap[e], G.Earap[e], 0.0);
    }
    double hS[kMfMaxS][2] = {{0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}};
    const int64_t o0 = G.mf_own_off[sl];
    const int no = G.mf_own_n[sl];
    for (int k = w; k < no; k += 4) {
        const int x = G.mf_own[(o0 + k) * 64 + lane];
        if (x < 0) continue;
        const int64_t e = x & ((1 << 27) - 1);
        const int ss = (x >> 27) & 7;
        if (!(x >> 30)) {
            add_rows(G.Jrep + 6 * e, 2, G.Wrep[e], G.Erep[2 * e], G.Erep[2 * e + 1]);
        } else {
            const double *J = G.Jdep + 4 * e;
            const double wv = G.Wdep[e], er = G.Edep[e];
            add_rows(J, 1, wv, er, 0.0);
#pragma unroll
            for (int q = 0; q < kMfMaxS; q++)
                if (q == ss - 1) { hS[q][0] += (J[3] * wv) * J[3]; hS[q][1] -= J[3] * (wv * er); }
        }
    }
#pragma unroll
    for (int q = 0; q < 12; q++) red[q][tid] = acc[q];
    __syncthreads();
    if (w == 0 && v >= 0) {
        double *D = G.mf_diag + G.moff[v];
        const int64_t o = G.voff[v];
#pragma unroll
        for (int q = 0; q < 12; q++) {
            const double t = (red[q][lane] + red[q][64 + lane]) + (red[q][128 + lane] + red[q][192 + lane]);
            if (q < 9) D[q] = t;
            else G.b[o + q - 9] = t;
        }
    }
    __syncthreads();
    // scale slots: diagonal entry and b part of the depth edges
    for (int j = 0; j < nh - nt; j++) {
        double h0 = 0.0, h1 = 0.0;
#pragma unroll
        for (int q = 0; q < kMfMaxS; q++)
            if (q == j) { h0 = hS[q][0]; h1 = hS[q][1]; }
        h0 = wave_sum(h0);
        h1 = wave_sum(h1);
        if (lane == 0) { red[0][w] = h0; red[1][w] = h1; }
        __syncthreads();
        if (tid < 2) {
            double *out = G.mf_hlin + G.hs_pos[G.sl_hoff[sl] + nt + j] * kMfLin;
            out[tid == 0 ? 0 : 21] = (red[tid][0] + red[tid][1]) + (red[tid][2] + red[tid][3]);
        }
        __syncthreads();
    }
}

// heavy rows: workgroup (heavy vertex, value) sums the value over the vertex's slot partials in
// position order (strided per thread, fixed tree); values 0..20 the lower 6 x 6 block, 21..26 b
__global__ void __launch_bounds__(256) k_mf_lin_heavy(const PcgDev G) {
    __shared__ double red[256];
    const int hk = blockIdx.x / kMfLin, q = blockIdx.x % kMfLin;
    const int v = G.heavy_v[hk], d = G.vdim[v];
    int a = 0, bcol = 0;
    if (q < 21) { while ((a + 1) * (a + 2) / 2 <= q) a++; bcol = q - a * (a + 1) / 2; if (a >= d) return; }
    else if (q - 21 >= d) return;
    const int64_t p0 = G.hv_slot_begin[hk], p1 = G.hv_slot_begin[hk + 1];
    double s = 0.0;
    for (int64_t p = p0 + threadIdx.x; p < p1; p += 256) s += G.mf_hlin[p * kMfLin + q];
    s = wg_tree(s, red);
    if (threadIdx.x == 0) {
        if (q < 21) {
            double *D = G.mf_diag + G.moff[v];
            D[a * d + bcol] = s;
            D[bcol * d + a] = s;
        } else {
            G.b[G.voff[v] + q - 21] = s;
        }
    }
}

// the diagonal of H per dof (for max diag)
__global__ void k_mf_dvec(const PcgDev G) {
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v >= G.nv) return;
    const int d = G.vdim[v];
    const double *D = G.mf_diag + G.moff[v];
    for (int i = 0; i < d; i++) G.mf_dvec[G.voff[v] + i] = D[i * d + i];
}

}  // namespace dev

void launch_pcg_repack(const PcgDev &G, const double *hval, hipStream_t st) {
    if (G.nslots + G.nhslots <= 0) return;
    hipEvent_t e0 = prof_begin(st);
    const unsigned grid = (unsigned)(((G.nslots + G.nhslots) * 64 + 255) / 256);
    hipLaunchKernelGGL(dev::k_pcg_repack, dim3(grid), dim3(256), 0, st, G, hval);
    prof_end("pcg_repack", e0, grid, 0.0, st);
}

void launch_mf_lin(const PcgDev &G, bool want_dvec, hipStream_t st) {
    if (G.nsl > 0) {
        hipEvent_t e0 = prof_begin(st);
        hipLaunchKernelGGL(dev::k_mf_lin, dim3(G.nsl), dim3(256), 0, st, G);
        prof_end("mf_lin", e0, G.nsl, 0.0, st);
    }
    if (G.nheavy > 0) {
        hipEvent_t e0 = prof_begin(st);
        hipLaunchKernelGGL(dev::k_mf_lin_heavy, dim3(G.nheavy * kMfLin), dim3(256), 0, st, G);
        prof_end("mf_lin_heavy", e0, G.nheavy * kMfLin, 0.0, st);
    }
    if (want_dvec && G.nv > 0)
        hipLaunchKernelGGL(dev::k_mf_dvec, dim3((unsigned)((G.nv + 255) / 256)), dim3(256), 0, st, G);
}

void launch_pcg_setup(const PcgDev &G, const double *hval, const double *b, double lambda, double *x,
                      hipStream_t st, bool rec_cleared) {
    if (!rec_cleared) hipMemsetAsync(G.rec, 0, sizeof(double) * kPcgRec * (size_t)(G.max_it + 2), st);
    if (G.nB <= 0) return;                             // (an empty problem: nothing to set up)
    hipEvent_t e0 = prof_begin(st);
    hipLaunchKernelGGL(dev::k_pcg_setup, dim3(G.nB), dim3(256), 0, st, G, hval, b, lambda, x);
    prof_end("pcg_setup", e0, G.nB, 0.0, st);
}

void launch_pcg_product(const PcgDev &G, int it, const double *hval, double lambda, hipStream_t st) {
    hipEvent_t e0 = prof_begin(st);
    // always launched (also with no slices): its workgroup 0 writes the iteration record
    const unsigned grid = (unsigned)std::max(G.nA_sl, 1);
    if (G.mf) {
        hipLaunchKernelGGL(dev::k_pcg_dots, dim3(1), dim3(256), 0, st, it, G);
        hipLaunchKernelGGL(dev::k_mf_product, dim3(grid), dim3(256), sizeof(double) * (size_t)G.mf_lds, st, it, G,
                           lambda);
    }
    else
        hipLaunchKernelGGL(dev::k_pcg_product, dim3(grid), dim3(256), 0, st, it, G, hval, lambda);
    prof_end("pcg_product", e0, grid, 0.0, st);
}

void launch_pcg_heavy(const PcgDev &G, int it, const double *hval, double lambda, hipStream_t st) {
    const unsigned grid = (unsigned)(G.nheavy_dofs + G.nA_light + (G.mf ? 1 : 0));
    if (grid == 0) return;
    hipEvent_t e0 = prof_begin(st);
    hipLaunchKernelGGL(dev::k_pcg_heavy, dim3(grid), dim3(256), 0, st, it, G, hval, lambda);
    prof_end("pcg_heavy", e0, grid, 0.0, st);
}

void launch_pcg_update(const PcgDev &G, int it, double lambda, double *x, hipStream_t st) {
    if (G.nB <= 0) return;
    hipEvent_t e0 = prof_begin(st);
    hipLaunchKernelGGL(dev::k_pcg_update, dim3(G.nB), dim3(256), 0, st, it, G, lambda, x);
    prof_end("pcg_update", e0, G.nB, 0.0, st);
}

// ---- host: the row view of the block structure ------------------------------------------------
bool build_pcg_host(int64_t nv, const std::vector<int64_t> &voff, const std::vector<int32_t> &vdim,
                    const std::vector<int64_t> &blk_val_off, const std::vector<int32_t> &blk_rows,
                    const std::vector<int32_t> &blk_cols, const std::vector<int64_t> &blk_row_dof,
                    const std::vector<int64_t> &blk_col_dof, const std::vector<int64_t> &elim_pos, PcgHost &H,
                    std::string &err) {
    H = PcgHost();
    const int64_t nb = (int64_t)blk_val_off.size();
    int64_t ndof = nv > 0 ? voff[nv - 1] + vdim[nv - 1] : 0;
    if (ndof >= (int64_t)INT32_MAX) { err = "pcg: dof count exceeds int32"; return false; }
    std::vector<int32_t> dof_v(std::max<int64_t>(ndof, 1), -1);
    for (int64_t v = 0; v < nv; v++) {
        if (vdim[v] < 1 || vdim[v] > 6) { err = "pcg: vertex dimension outside 1..6"; return false; }
        for (int k = 0; k < vdim[v]; k++) dof_v[voff[v] + k] = (int32_t)v;
    }
    std::vector<int64_t> cnt(nv + 1, 0);
    H.diag_off.assign(nv, -1);
    for (int64_t b = 0; b < nb; b++) {
        const int32_t rv = dof_v[blk_row_dof[b]], cv = dof_v[blk_col_dof[b]];
        if (rv < 0 || cv < 0) { err = "pcg: block outside the dof range"; return false; }
        cnt[rv]++;
        if (rv != cv) cnt[cv]++;
        else H.diag_off[rv] = blk_val_off[b];
    }
    H.ent_begin.assign(nv + 1, 0);
    for (int64_t v = 0; v < nv; v++) {
        if (H.diag_off[v] < 0) { err = "pcg: vertex without a diagonal block"; return false; }
        H.ent_begin[v + 1] = H.ent_begin[v] + cnt[v];
    }
    H.ent.resize(H.ent_begin[nv]);
    std::vector<int64_t> fill(H.ent_begin.begin(), H.ent_begin.end() - 1);
    for (int64_t b = 0; b < nb; b++) {
        const int32_t rv = dof_v[blk_row_dof[b]], cv = dof_v[blk_col_dof[b]];
        H.ent[fill[rv]++] = PcgEnt{blk_val_off[b], (int32_t)blk_col_dof[b], (int16_t)blk_cols[b], 0};
        if (rv != cv) H.ent[fill[cv]++] = PcgEnt{blk_val_off[b], (int32_t)blk_row_dof[b], (int16_t)blk_rows[b], 1};
    }
    for (int64_t v = 0; v < nv; v++)
        std::sort(H.ent.begin() + H.ent_begin[v], H.ent.begin() + H.ent_begin[v + 1],
                  [](const PcgEnt &a, const PcgEnt &b) { return a.odof < b.odof; });
    H.v_heavy.assign(nv, -1);
    H.h_first.push_back(0);
    H.h_dofbase.push_back(0);
    const int64_t chunk = kPcgChunk;
    std::vector<int32_t> sliced;
    for (int64_t v = 0; v < nv; v++) {
        const int64_t n = H.ent_begin[v + 1] - H.ent_begin[v];
        if (n > kPcgHeavy) {
            H.v_heavy[v] = (int32_t)H.heavy_v.size();
            H.heavy_v.push_back((int32_t)v);
            H.h_dofbase.push_back(H.h_dofbase.back() + vdim[v]);
        } else if (vdim[v] == 3) {
            sliced.push_back((int32_t)v);
        } else {
            H.light_v.push_back((int32_t)v);
        }
    }
    if (H.h_dofbase.back() > kPcgMaxHeavyDofs) { err = "pcg: too many heavy-row dofs"; return false; }
    std::vector<char> is_sliced(nv, 0);
    for (int32_t v : sliced) is_sliced[v] = 1;
    // heavy rows: the entries whose other vertex is not a sliced row stay as entries, in chunks (the
    // sliced rows' couplings to heavy vertices come back as per-slice reductions)
    H.hres.clear();
    for (int32_t hk = 0; hk < (int32_t)H.heavy_v.size(); hk++) {
        const int32_t v = H.heavy_v[hk];
        const int64_t b0 = (int64_t)H.hres.size();
        for (int64_t e = H.ent_begin[v]; e < H.ent_begin[v + 1]; e++) {
            const int32_t u = dof_v[H.ent[e].odof];
            if (!is_sliced[u]) H.hres.push_back(H.ent[e]);
        }
        const int64_t b1 = (int64_t)H.hres.size();
        for (int64_t e = b0; e < b1; e += chunk) {
            H.hc_vertex.push_back(hk);
            H.hc_beg.push_back(e);
            H.hc_end.push_back(std::min<int64_t>(e + chunk, b1));
        }
        H.h_first.push_back((int32_t)H.hc_vertex.size());
    }
    // sliced rows: nested-dissection order, by descending count of 3x3 blocks inside each window
    // (ties in that order), 64 per slice.  A row's entries: 3x3 blocks to light points -> 3x3 slots;
    // blocks to heavy vertices -> heavy slots (one per heavy vertex the slice couples to, shared by
    // its lanes); the rest -> extra entries
    auto cls = [&](const PcgEnt &E) {      // 0: 3x3 slot, 1: heavy slot, 2: extra entry
        const int32_t u = dof_v[E.odof];
        if (H.v_heavy[u] >= 0) return 1;
        return E.odim == 3 ? 0 : 2;
    };
    std::vector<int64_t> cnt3(nv, 0), cntx(nv, 0);
    for (int32_t v : sliced)
        for (int64_t e = H.ent_begin[v]; e < H.ent_begin[v + 1]; e++) {
            const int c = cls(H.ent[e]);
            cnt3[v] += c == 0;
            cntx[v] += c == 2;
        }
    std::sort(sliced.begin(), sliced.end(), [&](int32_t a, int32_t b) { return elim_pos[a] < elim_pos[b]; });
    for (size_t w = 0; w < sliced.size(); w += kPcgSortWindow)
        std::stable_sort(sliced.begin() + w, sliced.begin() + std::min(sliced.size(), w + kPcgSortWindow),
                         [&](int32_t a, int32_t b) { return cnt3[a] > cnt3[b]; });
    const int64_t nsl = ((int64_t)sliced.size() + 63) / 64;
    // XCD-aware slice order.  The product's workgroup b takes slice b, and workgroups b and b + 8 run
    // on one XCD (its own 4 MiB L2).  The 64-row groups of the nested-dissection order are dealt so
    // that each XCD's slices (b = x mod 8) are one contiguous run of that order: a slice's neighbour
    // (z, p_prev) gathers then hit lines its XCD's L2 already holds instead of every XCD fetching
    // the whole vector.
    std::vector<int32_t> rows(nsl * 64, -1);
    {
        const int nx = nsl >= 16 ? 8 : 1;
        std::vector<int64_t> start(nx + 1, 0);
        for (int x = 0; x < nx; x++) start[x + 1] = start[x] + (nsl - x + nx - 1) / nx;
        for (int64_t b = 0; b < nsl; b++) {
            const int64_t g = start[b % nx] + b / nx;         // spatial group of slice b
            for (int l = 0; l < 64 && g * 64 + l < (int64_t)sliced.size(); l++) rows[b * 64 + l] = sliced[g * 64 + l];
        }
    }
    H.sl_v.assign(nsl * 64, -1);
    H.sl_n.resize(nsl); H.sl_nx.resize(nsl); H.sl_off.resize(nsl); H.sl_xoff.resize(nsl);
    H.sl_hn.resize(nsl); H.sl_hoff.resize(nsl);
    std::vector<std::vector<int32_t>> sl_heavy(nsl);        // heavy vertices each slice couples to
    int64_t slots = 0, xslots = 0, hslots = 0;
    for (int64_t sl = 0; sl < nsl; sl++) {
        int64_t mn = 0, mx = 0;
        for (int l = 0; l < 64; l++) {
            const int32_t v = rows[sl * 64 + l];
            if (v < 0) continue;
            H.sl_v[sl * 64 + l] = v;
            mn = std::max(mn, cnt3[v]);
            mx = std::max(mx, cntx[v]);
            for (int64_t e = H.ent_begin[v]; e < H.ent_begin[v + 1]; e++)
                if (cls(H.ent[e]) == 1) sl_heavy[sl].push_back(H.v_heavy[dof_v[H.ent[e].odof]]);
        }
        std::sort(sl_heavy[sl].begin(), sl_heavy[sl].end());
        sl_heavy[sl].erase(std::unique(sl_heavy[sl].begin(), sl_heavy[sl].end()), sl_heavy[sl].end());
        H.sl_n[sl] = (int32_t)mn; H.sl_nx[sl] = (int32_t)mx; H.sl_hn[sl] = (int32_t)sl_heavy[sl].size();
        H.sl_off[sl] = slots; H.sl_xoff[sl] = xslots; H.sl_hoff[sl] = hslots;
        slots += mn; xslots += mx; hslots += (int64_t)sl_heavy[sl].size();
    }
    H.sl_map.assign(slots * 64, -1);
    H.sl_col.assign(slots * 64, 0);
    H.sl_x.assign(xslots * 64, PcgEnt{0, 0, 0, 0});
    H.hs_map.assign(hslots * 64, -1);
    H.hs_hk.resize(hslots);
    H.hs_voff.resize(hslots);
    for (int64_t sl = 0; sl < nsl; sl++) {
        for (size_t k = 0; k < sl_heavy[sl].size(); k++) H.hs_hk[H.sl_hoff[sl] + k] = sl_heavy[sl][k];
        for (int l = 0; l < 64; l++) {
            const int32_t v = H.sl_v[sl * 64 + l];
            if (v < 0) continue;
            int64_t k3 = 0, kx = 0;
            for (int64_t e = H.ent_begin[v]; e < H.ent_begin[v + 1]; e++) {
                const PcgEnt &E = H.ent[e];
                const int c = cls(E);
                if (c == 0) {
                    const int64_t g = H.sl_off[sl] + k3++;
                    H.sl_map[g * 64 + l] = E.val_off | ((int64_t)(E.tr ? 1 : 0) << 62);
                    H.sl_col[g * 64 + l] = E.odof;
                } else if (c == 1) {
                    const int32_t hk = H.v_heavy[dof_v[E.odof]];
                    const auto it = std::lower_bound(sl_heavy[sl].begin(), sl_heavy[sl].end(), hk);
                    const int64_t g = H.sl_hoff[sl] + (it - sl_heavy[sl].begin());
                    if (H.hs_map[g * 64 + l] != -1) { err = "pcg: two blocks between one row and one heavy vertex"; return false; }
                    H.hs_map[g * 64 + l] = E.val_off | ((int64_t)(E.tr ? 1 : 0) << 62);
                } else {
                    H.sl_x[(H.sl_xoff[sl] + kx++) * 64 + l] = E;
                }
            }
        }
    }
    int64_t hsv = 0, hs_bytes = 0;
    for (int64_t g = 0; g < hslots; g++) {
        const int od = vdim[H.heavy_v[H.hs_hk[g]]];
        const int nq = od == 1 ? 2 : 5 * ((od + 2) / 3);
        H.hs_voff[g] = hsv;
        hsv += 64 * (int64_t)nq;
        hs_bytes += 64 * 16 * (int64_t)nq;
    }
    H.hs_size = 2 * hsv;
    // per heavy vertex: its slots, ascending (the order its row sums their partials in); a slot's
    // partial lands at its position in that order
    H.hv_slot_begin.assign(H.heavy_v.size() + 1, 0);
    for (int64_t g = 0; g < hslots; g++) H.hv_slot_begin[H.hs_hk[g] + 1]++;
    for (size_t k = 0; k < H.heavy_v.size(); k++) H.hv_slot_begin[k + 1] += H.hv_slot_begin[k];
    H.hs_pos.resize(hslots);
    {
        std::vector<int64_t> f(H.hv_slot_begin.begin(), H.hv_slot_begin.end() - 1);
        for (int64_t g = 0; g < hslots; g++) H.hs_pos[g] = f[H.hs_hk[g]]++;
    }
    // bytes a product launch loads / stores apart from the neighbours' (z, p_prev) gathers: own
    // (z, p_prev) read and (p, q) written, repacked 3x3 slots with column indices and heavy slots
    // (padding included), the extra entries with their blocks, the generic rows' and heavy rows'
    // remaining entries with their blocks; flops: 2 per block entry of H
    {
        int64_t ndof_ = nv > 0 ? voff[nv - 1] + vdim[nv - 1] : 0;
        double by = 32.0 * (double)ndof_ + 64.0 * 80.0 * (double)slots + (double)hs_bytes +
                    16.0 * (double)H.sl_x.size() + 8.0 * 6.0 * (double)hslots;
        double fl = 0;
        for (int64_t v = 0; v < nv; v++)
            for (int64_t e = H.ent_begin[v]; e < H.ent_begin[v + 1]; e++) {
                const PcgEnt &E = H.ent[e];
                fl += 2.0 * vdim[v] * E.odim;
                if (is_sliced[v]) { if (cls(E) == 2) by += 8.0 * 3 * E.odim; continue; }
                if (H.v_heavy[v] >= 0 && is_sliced[dof_v[E.odof]]) continue;   // via the heavy slots
                by += 16.0 + 8.0 * vdim[v] * E.odim;
            }
        H.product_bytes = by;
        H.product_flops = fl;
    }
    H.moff.resize(nv);
    for (int64_t v = 0; v < nv; v++) { H.moff[v] = H.msize; H.msize += (int64_t)vdim[v] * vdim[v]; }
    return true;
}

// ---- host: the matrix-free plan -----------------------------------------------------------------
bool build_pcg_mf(int64_t nv, const std::vector<int64_t> &voff, const std::vector<int32_t> &vdim,
                  const std::vector<int64_t> &elim_pos, int Q, int S, int R, int D, int E,
                  const int32_t *rep_point, const int32_t *dep_point, const int32_t *dep_scale,
                  const int32_t *arap_pts, const int32_t *arap_pair, PcgMfHost &H, std::string &err) {
    H = PcgMfHost();
    const int64_t ndof = nv > 0 ? voff[nv - 1] + vdim[nv - 1] : 0;
    if (ndof >= (int64_t)INT32_MAX) { err = "dof count exceeds int32"; return false; }
    const int64_t P = nv - Q - S;
    if (P < 0) { err = "vertex count below pairs + scales"; return false; }
    auto vP = [&](int64_t p) { return (int64_t)Q + S + p; };
    // vertex classes: 3-dof points are sliced rows; every other vertex (T_g, scales) a heavy row
    H.v_heavy.assign(nv, -1);
    H.h_dofbase.push_back(0);
    std::vector<int32_t> sliced;
    for (int64_t v = 0; v < nv; v++) {
        if (vdim[v] < 1 || vdim[v] > 6) { err = "vertex dimension outside 1..6"; return false; }
        if (v >= (int64_t)Q + S && vdim[v] == 3) {
            sliced.push_back((int32_t)v);
        } else {
            H.v_heavy[v] = (int32_t)H.heavy_v.size();
            H.heavy_v.push_back((int32_t)v);
            H.h_dofbase.push_back(H.h_dofbase.back() + vdim[v]);
        }
    }
    if (H.h_dofbase.back() > kPcgMaxHeavyDofs) { err = "too many heavy-row dofs"; return false; }
    H.h_first.assign(H.heavy_v.size() + 1, 0);
    for (int i = 0; i < P; i++)
        if (vdim[vP(i)] != 3) { err = "point vertex not 3-dof"; return false; }
    // rows: the copies of one mesh vertex (the points an ARAP edge pairs at roles (0, 1) and (2, 3):
    // the same vertex in the pair's two keyframes) kept together, groups in nested-dissection order
    // (a group at its first member's position), 64 rows per slice, dealt to XCDs in contiguous runs
    // (as build_pcg_host).  Every ARAP edge then touches one copy group per mesh vertex, so a slice
    // holds most of its edges' roles and few edges are loaded by two slices.
    auto pidx = [&](int32_t v) { return (int64_t)v - Q - S; };
    std::vector<int32_t> grp(P);
    for (int64_t i = 0; i < P; i++) grp[i] = (int32_t)i;
    auto find = [&](int32_t x) {
        while (grp[x] != x) { grp[x] = grp[grp[x]]; x = grp[x]; }
        return x;
    };
    for (int64_t e = 0; e < E; e++)
        for (int r = 0; r < 4; r += 2) {
            const int32_t a = find(arap_pts[4 * e + r]), b = find(arap_pts[4 * e + r + 1]);
            if (a != b) grp[std::max(a, b)] = std::min(a, b);
        }
    std::vector<int64_t> gpos(P, INT64_MAX);
    for (int64_t i = 0; i < P; i++) {
        const int32_t g = find((int32_t)i);
        gpos[g] = std::min(gpos[g], elim_pos[vP(i)]);
    }
    std::sort(sliced.begin(), sliced.end(), [&](int32_t a, int32_t b) {
        const int64_t ga = gpos[find((int32_t)pidx(a))], gb = gpos[find((int32_t)pidx(b))];
        return ga != gb ? ga < gb : elim_pos[a] < elim_pos[b];
    });
    const int64_t nsl = ((int64_t)sliced.size() + 63) / 64;
    H.sl_v.assign(nsl * 64, -1);
    {
        const int nx = nsl >= 16 ? 8 : 1;
        std::vector<int64_t> start(nx + 1, 0);
        for (int x = 0; x < nx; x++) start[x + 1] = start[x] + (nsl - x + nx - 1) / nx;
        for (int64_t b = 0; b < nsl; b++) {
            const int64_t g = start[b % nx] + b / nx;
            for (int l = 0; l < 64 && g * 64 + l < (int64_t)sliced.size(); l++) H.sl_v[b * 64 + l] = sliced[g * 64 + l];
        }
    }
    std::vector<int32_t> pslice(P, -1), plane(P, -1);
    for (int64_t sl = 0; sl < nsl; sl++)
        for (int l = 0; l < 64; l++) {
            const int32_t v = H.sl_v[sl * 64 + l];
            if (v >= 0) { pslice[pidx(v)] = (int32_t)sl; plane[pidx(v)] = l; }
        }
    // per slice: its local edges (an edge is listed by every slice holding one of its points)
    std::vector<std::vector<int64_t>> sl_edges(nsl);      // kind << 40 | edge
    auto add_local = [&](int kind, int64_t e, const int32_t *pts, int np) {
        int32_t seen[4];
        int ns = 0;
        for (int r = 0; r < np; r++) {
            const int32_t s0 = pslice[pts[r]];
            bool dup = false;
            for (int q = 0; q < ns; q++) dup |= seen[q] == s0;
            if (!dup) { seen[ns++] = s0; sl_edges[s0].push_back(((int64_t)kind << 40) | e); }
        }
    };
    if ((int64_t)E >= (1LL << 40) || kMfMaxLds > 0x7fff || kMfMaxT > 7 || kMfMaxS > 7 || R >= (1 << 27) ||
        D >= (1 << 27)) {
        err = "record fields overflow";
        return false;
    }
    for (int64_t e = 0; e < E; e++) add_local(MF_ARAP, e, arap_pts + 4 * e, 4);
    // the points' single-point edges (their own lane sums them): CSR by point, edges ascending
    std::vector<int64_t> own_beg(P + 1, 0);
    for (int e = 0; e < R; e++) own_beg[rep_point[e] + 1]++;
    for (int e = 0; e < D; e++) own_beg[dep_point[e] + 1]++;
    for (int64_t i = 0; i < P; i++) own_beg[i + 1] += own_beg[i];
    std::vector<int32_t> own_e(own_beg[P]);      // MF_REP / MF_DEP << 30 | edge
    {
        std::vector<int64_t> f(own_beg.begin(), own_beg.end() - 1);
        for (int e = 0; e < R; e++) own_e[f[rep_point[e]]++] = e;
        for (int e = 0; e < D; e++) own_e[f[dep_point[e]]++] = (1 << 30) | e;
    }
    H.le_off.resize(nsl); H.le_n.resize(nsl); H.le_na.resize(nsl);
    H.in_off.resize(nsl); H.in_n.resize(nsl); H.sl_hn.resize(nsl); H.sl_nt.resize(nsl); H.sl_hoff.resize(nsl);
    H.own_off.resize(nsl); H.own_n.resize(nsl);
    int64_t nle = 0, nin = 0, hslots = 0;
    std::vector<std::vector<int32_t>> sl_heavy(nsl);
    auto owner = [&](int64_t e) -> int32_t {     // of an ARAP edge: the first slice holding one of its points
        int32_t o = INT32_MAX;
        for (int r = 0; r < 4; r++) o = std::min(o, pslice[arap_pts[4 * e + r]]);
        return o;
    };
    // per slice: heavy slots = the T_g of its owned ARAP edges (first: T_g vertices precede the
    // scales in vertex order), then the scales of its points' depth edges
    std::vector<std::vector<int32_t>> sl_scales(nsl);
    int64_t nown = 0;
    for (int64_t sl = 0; sl < nsl; sl++) {
        auto &L = sl_edges[sl];
        std::sort(L.begin(), L.end());
        for (int64_t x : L) {
            const int64_t e = x & 0xffffffffffLL;
            if (owner(e) == sl) sl_heavy[sl].push_back(H.v_heavy[arap_pair[e]]);
        }
        std::sort(sl_heavy[sl].begin(), sl_heavy[sl].end());
        sl_heavy[sl].erase(std::unique(sl_heavy[sl].begin(), sl_heavy[sl].end()), sl_heavy[sl].end());
        const int nt = (int)sl_heavy[sl].size();
        int64_t mo = 0;
        for (int l = 0; l < 64; l++) {
            const int32_t v = H.sl_v[sl * 64 + l];
            if (v < 0) continue;
            const int64_t p = pidx(v);
            mo = std::max(mo, own_beg[p + 1] - own_beg[p]);
            for (int64_t k = own_beg[p]; k < own_beg[p + 1]; k++)
                if (own_e[k] >> 30) sl_scales[sl].push_back(H.v_heavy[(int64_t)Q + dep_scale[own_e[k] & ((1 << 30) - 1)]]);
        }
        std::sort(sl_scales[sl].begin(), sl_scales[sl].end());
        sl_scales[sl].erase(std::unique(sl_scales[sl].begin(), sl_scales[sl].end()), sl_scales[sl].end());
        if (nt > kMfMaxT || (int)sl_scales[sl].size() > kMfMaxS) {
            err = "a slice couples to more global vertices than the kernels' accumulators";
            return false;
        }
        sl_heavy[sl].insert(sl_heavy[sl].end(), sl_scales[sl].begin(), sl_scales[sl].end());
        int64_t lds = 0;                      // one 3-vector per (local edge, role in this slice)
        for (int64_t x : L) {
            const int64_t e = x & 0xffffffffffLL;
            for (int r = 0; r < 4; r++) lds += 3 * (pslice[arap_pts[4 * e + r]] == sl);
        }
        if (lds > kMfMaxLds) { err = "a slice's local edges exceed the LDS budget"; return false; }
        H.max_lds = std::max<int32_t>(H.max_lds, (int32_t)lds);
        H.le_off[sl] = nle; H.le_n[sl] = (int32_t)L.size(); H.le_na[sl] = (int32_t)L.size();
        H.sl_hn[sl] = (int32_t)sl_heavy[sl].size(); H.sl_nt[sl] = nt; H.sl_hoff[sl] = hslots;
        H.own_off[sl] = nown; H.own_n[sl] = (int32_t)mo;
        nle += (int64_t)L.size();
        nown += mo;
        hslots += (int64_t)sl_heavy[sl].size();
    }
    H.own.assign((size_t)nown * 64, -1);
    H.le.resize(nle);
    H.hs_hk.resize(hslots);
    // incidences: per row, (local edge, role) in local-edge order
    std::vector<std::vector<int32_t>> rowinc(64), rowinc2(64);
    for (int64_t sl = 0; sl < nsl; sl++) {
        const auto &L = sl_edges[sl];
        for (size_t k = 0; k < sl_heavy[sl].size(); k++) H.hs_hk[H.sl_hoff[sl] + k] = sl_heavy[sl][k];
        for (auto &r : rowinc) r.clear();
        for (auto &r : rowinc2) r.clear();
        int32_t base = 0;
        for (size_t k = 0; k < L.size(); k++) {
            const int kind = (int)(L[k] >> 40);
            const int64_t e = L[k] & 0xffffffffffLL;
            int64_t hs = 0;                   // T_g slot (+1) of an owned edge
            if (owner(e) == sl)
                hs = 1 + (std::find(sl_heavy[sl].begin(), sl_heavy[sl].begin() + H.sl_nt[sl], H.v_heavy[arap_pair[e]]) -
                          sl_heavy[sl].begin());
            int64_t mask = 0;
            const int32_t b0 = base;
            for (int r = 0; r < 4; r++) {
                const int32_t p = arap_pts[4 * e + r];
                if (pslice[p] != sl) continue;
                mask |= 1LL << r;
                rowinc[plane[p]].push_back(base);
                rowinc2[plane[p]].push_back(((int32_t)k << 2) | r);
                base += 3;
            }
            H.le[H.le_off[sl] + k] = ((int64_t)kind << 62) | (mask << 58) | (hs << 55) | ((int64_t)b0 << 40) | e;
        }
        size_t mx = 0;
        for (const auto &r : rowinc) mx = std::max(mx, r.size());
        H.in_off[sl] = nin; H.in_n[sl] = (int32_t)mx;
        H.inc.resize((size_t)(nin + (int64_t)mx) * 64, -1);
        H.inc2.resize((size_t)(nin + (int64_t)mx) * 64, -1);
        for (int l = 0; l < 64; l++)
            for (size_t k = 0; k < rowinc[l].size(); k++) {
                H.inc[(nin + (int64_t)k) * 64 + l] = rowinc[l][k];
                H.inc2[(nin + (int64_t)k) * 64 + l] = rowinc2[l][k];
            }
        nin += (int64_t)mx;
        // own edges: per lane in point-edge order; depth edges carry their scale slot (+1)
        for (int l = 0; l < 64; l++) {
            const int32_t v = H.sl_v[sl * 64 + l];
            if (v < 0) continue;
            const int64_t p = pidx(v);
            for (int64_t k = own_beg[p]; k < own_beg[p + 1]; k++) {
                int32_t x = own_e[k];
                if (x >> 30) {
                    const int32_t hk = H.v_heavy[(int64_t)Q + dep_scale[x & ((1 << 30) - 1)]];
                    const int32_t j = (int32_t)(std::lower_bound(sl_scales[sl].begin(), sl_scales[sl].end(), hk) -
                                                sl_scales[sl].begin());
                    x |= (j + 1) << 27;
                }
                H.own[(H.own_off[sl] + (k - own_beg[p])) * 64 + l] = x;
            }
        }
    }
    H.hv_slot_begin.assign(H.heavy_v.size() + 1, 0);
    for (int64_t g = 0; g < hslots; g++) H.hv_slot_begin[H.hs_hk[g] + 1]++;
    for (size_t k = 0; k < H.heavy_v.size(); k++) H.hv_slot_begin[k + 1] += H.hv_slot_begin[k];
    H.hs_pos.resize(hslots);
    {
        std::vector<int64_t> f(H.hv_slot_begin.begin(), H.hv_slot_begin.end() - 1);
        for (int64_t g = 0; g < hslots; g++) H.hs_pos[g] = f[H.hs_hk[g]]++;
    }
    // per slice: one 32-byte metadata record (the product reads it with two 16-byte loads) and the
    // partial positions of its heavy slots
    H.sl_meta.assign(4 * (size_t)nsl, 0);
    H.sl_hpos.assign((size_t)nsl * kMfMaxH, 0);
    for (int64_t sl = 0; sl < nsl; sl++) {
        if (H.le_n[sl] > 0xffff || H.in_n[sl] > 0xff || H.own_n[sl] > 0xff || H.sl_hn[sl] > kMfMaxH) {
            err = "slice metadata fields overflow";
            return false;
        }
        H.sl_meta[4 * sl] = H.le_off[sl];
        H.sl_meta[4 * sl + 1] = H.in_off[sl];
        H.sl_meta[4 * sl + 2] = H.own_off[sl];
        H.sl_meta[4 * sl + 3] = (int64_t)H.le_n[sl] | ((int64_t)H.in_n[sl] << 16) | ((int64_t)H.own_n[sl] << 24) |
                                ((int64_t)H.sl_nt[sl] << 32) | ((int64_t)H.sl_hn[sl] << 36);
        for (int h = 0; h < H.sl_hn[sl]; h++) H.sl_hpos[sl * kMfMaxH + h] = (int32_t)H.hs_pos[H.sl_hoff[sl] + h];
    }
    // the edges' vertex dofs
    H.adof.resize(4 * (size_t)E); H.atdof.resize(E); H.rdof.resize(R); H.ddof.resize(2 * (size_t)D);
    for (int64_t e = 0; e < E; e++) {
        for (int r = 0; r < 4; r++) H.adof[4 * e + r] = (int32_t)voff[vP(arap_pts[4 * e + r])];
        H.atdof[e] = (int32_t)voff[arap_pair[e]];
    }
    for (int e = 0; e < R; e++) H.rdof[e] = (int32_t)voff[vP(rep_point[e])];
    for (int e = 0; e < D; e++) {
        H.ddof[2 * e] = (int32_t)voff[vP(dep_point[e])];
        H.ddof[2 * e + 1] = (int32_t)voff[(int64_t)Q + dep_scale[e]];
    }
    H.moff.resize(nv);
    for (int64_t v = 0; v < nv; v++) { H.moff[v] = H.msize; H.msize += (int64_t)vdim[v] * vdim[v]; }
    // bytes one product launch loads / stores apart from the edges' (z, p_prev) gathers: per local
    // edge its record, Jacobian, weight and vertex dofs (an edge touching k slices counted k times),
    // the incidence slots, own (z, p_prev) read and (p, q) written, heavy partials; flops: 2 per
    // Jacobian entry for J p and J^T s
    {
        // per ARAP local edge: record 8 + J 144 + W 8 + dofs 20; per own edge: reprojection J 48 +
        // W 8, depth J 32 + W 8 + scale dof 4; slot entries 4 B per lane
        double by = 32.0 * (double)ndof + 4.0 * 64.0 * (double)(nin + nown) + 48.0 * (double)hslots, fl = 0;
        by += (double)nle * (8 + 144 + 8 + 20) + (double)R * (48 + 8) + (double)D * (32 + 8 + 4);
        fl += 4.0 * 18 * (double)nle + 4.0 * 6 * R + 4.0 * 4 * D;
        H.product_bytes = by;
        H.product_flops = fl;
    }
    return true;
}

}  // namespace deftri
