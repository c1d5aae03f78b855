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
#include <string>

#include "kernels.h"
#include "pcg.h"

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
__device__ __forceinline__ double pval(const double *__restrict__ z, const double *__restrict__ pp, double beta,
                                       int64_t i) {
    return __fma_rn(beta, pp[i], z[i]);
}

// acc[0..d) += B p_other for one entry of the row (B the block in this row's orientation)
__device__ __forceinline__ void ent_acc(const PcgEnt &E, int d, const double *__restrict__ hval,
                                        const double *__restrict__ z, const double *__restrict__ pp, double beta,
                                        double acc[6]) {
    const double *h = hval + E.val_off;
    const int od = E.odim;
    double pj[6];
#pragma unroll
    for (int j = 0; j < 6; j++) pj[j] = j < od ? pval(z, pp, beta, E.odof + j) : 0.0;
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
#pragma unroll
        for (int i = 0; i < 6; i++) {
            if (i < d) {
                double zi = 0.0;
#pragma unroll
                for (int j = 0; j < 6; j++)
                    if (j < d) zi += Mi[i * 6 + j] * rv[j];
                G.r[o + i] = rv[i];
                G.z[o + i] = zi;
                G.p[0][o + i] = 0.0;
                G.p[1][o + i] = 0.0;
                x[o + i] = 0.0;
                rz += rv[i] * zi;
                rr += rv[i] * rv[i];
            }
        }
    }
    red[0][threadIdx.x] = rz;
    red[1][threadIdx.x] = rr;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) {
            red[0][threadIdx.x] += red[0][threadIdx.x + off];
            red[1][threadIdx.x] += red[1][threadIdx.x + off];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) { G.partB[2 * blockIdx.x] = red[0][0]; G.partB[2 * blockIdx.x + 1] = red[1][0]; }
}

__global__ void __launch_bounds__(256) k_pcg_product(int it, const PcgDev G, const double *__restrict__ hval,
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
    const double *pp = G.p[it & 1];
    double *pn = G.p[(it + 1) & 1];
    const double *z = G.z;
    if ((int)blockIdx.x < G.nA_light) {
        const int k = blockIdx.x * 256 + tid;
        double pq = 0.0;
        if (k < G.nlight) {
            const int v = G.light_v[k];
            const int d = G.vdim[v];
            const int64_t o = G.voff[v];
            double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
            const int64_t e1 = G.ent_begin[v + 1];
            for (int64_t e = G.ent_begin[v]; e < e1; e++) ent_acc(load_ent(G.ent, e), d, hval, z, pp, beta, acc);
#pragma unroll
            for (int i = 0; i < 6; i++) {
                if (i < d) {
                    const double pv = pval(z, pp, beta, o + i);
                    const double qv = acc[i] + lam * pv;
                    pn[o + i] = pv;
                    G.q[o + i] = qv;
                    pq += pv * qv;
                }
            }
        }
        const double s = wg_tree(pq, red[0]);
        if (tid == 0) G.partA[blockIdx.x] = s;
        return;
    }
    // a chunk of a heavy row: partial sums of its entries, reduced in a fixed tree
    const int c = blockIdx.x - G.nA_light;
    const int hk = G.hc_vertex[c];
    const int v = G.heavy_v[hk];
    const int d = G.vdim[v];
    double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    const int64_t e1 = G.hc_end[c];
    for (int64_t e = G.hc_beg[c] + tid; e < e1; e += 256) ent_acc(load_ent(G.ent, e), d, hval, z, pp, beta, acc);
#pragma unroll
    for (int i = 0; i < 6; i++) red[i][tid] = acc[i];
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (tid < off)
#pragma unroll
            for (int i = 0; i < 6; i++) red[i][tid] += red[i][tid + off];
        __syncthreads();
    }
    if (tid < d) {
        G.hq[6 * c + tid] = red[tid][0];
        if (c == G.h_first[hk]) {
            const int64_t o = G.voff[v];
            pn[o + tid] = pval(z, pp, beta, o + tid);
        }
    }
}

__global__ void __launch_bounds__(256) k_pcg_update(int it, const PcgDev G, double lam, double *__restrict__ x) {
    __shared__ double red[2][256];
    __shared__ double hqs[kPcgMaxHeavyDofs];
    __shared__ double hps[kPcgMaxHeavyDofs];
    double *rec = G.rec + kPcgRec * (it + 1);
    if (rec[PR_STATUS] != 0.0) return;
    const int tid = threadIdx.x;
    const double *pn = G.p[(it + 1) & 1];
    const double pq_light = wg_tree([&] {
        double a = 0.0;
        for (int i = tid; i < G.nA_light; i += 256) a += G.partA[i];
        return a;
    }(), red[0]);
    // the heavy rows: chunk partials summed in chunk order, + lambda p
    for (int k = tid; k < G.nheavy_dofs; k += 256) {
        int hk = 0;
        while (G.h_dofbase[hk + 1] <= k) hk++;
        const int i = k - G.h_dofbase[hk];
        double s = 0.0;
        for (int c = G.h_first[hk]; c < G.h_first[hk + 1]; c++) s += G.hq[6 * c + i];
        const double pv = pn[G.voff[G.heavy_v[hk]] + i];
        hqs[k] = s + lam * pv;
        hps[k] = pv;
    }
    __syncthreads();
    if (tid == 0) {
        double a = 0.0;
        for (int k = 0; k < G.nheavy_dofs; k++) a += hps[k] * hqs[k];
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
        double rv[6];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            rv[i] = 0.0;
            if (i < d) {
                const double qv = hk < 0 ? G.q[o + i] : hqs[G.h_dofbase[hk] + i];
                x[o + i] += alpha * pn[o + i];
                rv[i] = G.r[o + i] - alpha * qv;
                G.r[o + i] = rv[i];
            }
        }
        const double *M = G.minv + G.moff[v];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            if (i < d) {
                double zi = 0.0;
#pragma unroll
                for (int j = 0; j < 6; j++)
                    if (j < d) zi += M[i * d + j] * rv[j];
                G.z[o + i] = zi;
                rz += rv[i] * zi;
                rr += rv[i] * rv[i];
            }
        }
    }
    red[0][tid] = rz;
    red[1][tid] = rr;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (tid < off) {
            red[0][tid] += red[0][tid + off];
            red[1][tid] += red[1][tid + off];
        }
        __syncthreads();
    }
    if (tid == 0) { G.partB[2 * blockIdx.x] = red[0][0]; G.partB[2 * blockIdx.x + 1] = red[1][0]; }
}

}  // namespace dev

void launch_pcg_setup(const PcgDev &G, const double *hval, const double *b, double lambda, double *x,
                      hipStream_t st) {
    hipMemsetAsync(G.rec, 0, sizeof(double) * kPcgRec * (size_t)(G.max_it + 2), st);
    hipEvent_t e0 = prof_begin(st);
    hipLaunchKernelGGL(dev::k_pcg_setup, dim3(G.nB), dim3(256), 0, st, G, hval, b, lambda, x);
    prof_end("pcg_setup", e0, G.nB, 0.0, st);
}

void launch_pcg_product(const PcgDev &G, int it, const double *hval, double lambda, hipStream_t st) {
    hipEvent_t e0 = prof_begin(st);
    hipLaunchKernelGGL(dev::k_pcg_product, dim3(G.nA_light + G.nhchunks), dim3(256), 0, st, it, G, hval, lambda);
    prof_end("pcg_product", e0, G.nA_light + G.nhchunks, 0.0, st);
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
                    const std::vector<int64_t> &blk_col_dof, PcgHost &H, std::string &err) {
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
    for (int64_t v = 0; v < nv; v++) {
        const int64_t n = H.ent_begin[v + 1] - H.ent_begin[v];
        if (n <= kPcgHeavy) { H.light_v.push_back((int32_t)v); continue; }
        const int32_t hk = (int32_t)H.heavy_v.size();
        H.v_heavy[v] = hk;
        H.heavy_v.push_back((int32_t)v);
        for (int64_t e = H.ent_begin[v]; e < H.ent_begin[v + 1]; e += kPcgChunk) {
            H.hc_vertex.push_back(hk);
            H.hc_beg.push_back(e);
            H.hc_end.push_back(std::min<int64_t>(e + kPcgChunk, H.ent_begin[v + 1]));
        }
        H.h_first.push_back((int32_t)H.hc_vertex.size());
        H.h_dofbase.push_back(H.h_dofbase.back() + vdim[v]);
    }
    if (H.h_dofbase.back() > kPcgMaxHeavyDofs) { err = "pcg: too many heavy-row dofs"; return false; }
    H.moff.resize(nv);
    for (int64_t v = 0; v < nv; v++) { H.moff[v] = H.msize; H.msize += (int64_t)vdim[v] * vdim[v]; }
    return true;
}

}  // namespace deftri
