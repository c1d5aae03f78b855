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
        const double *D = hval + G.diag_off[v];
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
        double rv[6], Mi[36];
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
                    if (i < d) { M[i * d + c] = y[i]; Mi[i * 6 + c] = y[i]; }
            }
        }
#pragma unroll
        for (int i = 0; i < 6; i++) rv[i] = i < d ? b[o + i] : 0.0;
        double2 *zp = reinterpret_cast<double2 *>(G.zp);
#pragma unroll
        for (int i = 0; i < 6; i++) {
            if (i < d) {
                double zi = 0.0;
#pragma unroll
                for (int j = 0; j < 6; j++)
                    if (j < d) zi += Mi[i * 6 + j] * rv[j];
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
    if (rec[PR_STATUS] != 0.0) return;
    const double beta = it == 0 ? 0.0 : rec[PR_RZ] / G.rec[kPcgRec * it + PR_RZ];
    const double *zp = G.zp;
    double2 *pq2 = reinterpret_cast<double2 *>(G.pq);
    const int tid = threadIdx.x;
    if ((int)blockIdx.x >= G.nheavy_dofs) {
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
    // four independent strided streams per thread (loads in flight together), combined in order
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    for (int64_t t = b0 + tid; t < b1; t += 1024)
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (t + 256 * u < b1) a[u] += G.hs_part[(t + 256 * u) * 6 + i];
    const double s_slots = wg_tree((a[0] + a[1]) + (a[2] + a[3]), red);
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
    if (rec[PR_STATUS] != 0.0) return;
    const int tid = threadIdx.x;
    const double2 *pq2 = reinterpret_cast<const double2 *>(G.pq);
    const int nA = G.nA_sl + G.nA_light;
    const double pq_light = wg_tree([&] {
        double a = 0.0;
        for (int i = tid; i < nA; i += 256) a += G.partA[i];
        return a;
    }(), red[0]);
    // the heavy rows' p.q (their q from k_pcg_heavy), in heavy-dof order
    if (tid == 0) {
        double a = 0.0;
        for (int hk = 0; hk < G.nheavy; hk++) {
            const int64_t o = G.voff[G.heavy_v[hk]];
            for (int i = 0; i < G.h_dofbase[hk + 1] - G.h_dofbase[hk]; i++) a += pq2[o + i].x * G.hqf[G.h_dofbase[hk] + i];
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
    const int64_t v = (int64_t)blockIdx.x * 256 + tid;
    double rz = 0.0, rr = 0.0;
    if (v < G.nv) {
        const int d = G.vdim[v];
        const int64_t o = G.voff[v];
        const int hk = G.v_heavy[v];
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

}  // namespace dev

void launch_pcg_repack(const PcgDev &G, const double *hval, hipStream_t st) {
    if (G.nslots + G.nhslots <= 0) return;
    hipEvent_t e0 = prof_begin(st);
    const unsigned grid = (unsigned)(((G.nslots + G.nhslots) * 64 + 255) / 256);
    hipLaunchKernelGGL(dev::k_pcg_repack, dim3(grid), dim3(256), 0, st, G, hval);
    prof_end("pcg_repack", e0, grid, 0.0, st);
}

void launch_pcg_setup(const PcgDev &G, const double *hval, const double *b, double lambda, double *x,
                      hipStream_t st) {
    hipMemsetAsync(G.rec, 0, sizeof(double) * kPcgRec * (size_t)(G.max_it + 2), st);
    hipEvent_t e0 = prof_begin(st);
    hipLaunchKernelGGL(dev::k_pcg_setup, dim3(G.nB), dim3(256), 0, st, G, hval, b, lambda, x);
    prof_end("pcg_setup", e0, G.nB, 0.0, st);
}

void launch_pcg_product(const PcgDev &G, int it, const double *hval, double lambda, hipStream_t st) {
    hipEvent_t e0 = prof_begin(st);
    // always launched (also with no slices): its workgroup 0 writes the iteration record
    const unsigned grid = (unsigned)std::max(G.nA_sl, 1);
    hipLaunchKernelGGL(dev::k_pcg_product, dim3(grid), dim3(256), 0, st, it, G, hval, lambda);
    prof_end("pcg_product", e0, grid, 0.0, st);
}

void launch_pcg_heavy(const PcgDev &G, int it, const double *hval, double lambda, hipStream_t st) {
    const unsigned grid = (unsigned)(G.nheavy_dofs + G.nA_light);
    if (grid == 0) return;
    hipEvent_t e0 = prof_begin(st);
    hipLaunchKernelGGL(dev::k_pcg_heavy, dim3(grid), dim3(256), 0, st, it, G, hval, lambda);
    prof_end("pcg_heavy", e0, grid, 0.0, st);
}

void launch_pcg_update(const PcgDev &G, int it, double lambda, double *x, hipStream_t st) {
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
    // A/B knobs (measurements in DESIGN.md): heavy-row chunk size, rows sliced or all generic
    static const int64_t chunk = [] { const char *e = std::getenv("DEFTRI_PCG_CHUNK"); return e ? std::max(64, std::atoi(e)) : kPcgChunk; }();
    static const bool no_slice = std::getenv("DEFTRI_PCG_NO_SLICE") != nullptr;
    std::vector<int32_t> sliced;
    for (int64_t v = 0; v < nv; v++) {
        const int64_t n = H.ent_begin[v + 1] - H.ent_begin[v];
        if (n > kPcgHeavy) {
            H.v_heavy[v] = (int32_t)H.heavy_v.size();
            H.heavy_v.push_back((int32_t)v);
            H.h_dofbase.push_back(H.h_dofbase.back() + vdim[v]);
        } else if (vdim[v] == 3 && !no_slice) {
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
        static const bool no_xcd = std::getenv("DEFTRI_PCG_NO_XCD") != nullptr;
        const int nx = (!no_xcd && nsl >= 16) ? 8 : 1;
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

}  // namespace deftri
