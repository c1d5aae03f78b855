// ba.hip — gfx950 kernels of the bundle-adjustment LM path (BlockSolver_6_3 Schur, reference
// g2oBundleAdjustment.cc:38-444; edge types g2oTypes.h:150-229, g2oTypes.cc:121-189).
//
// Stage (g2o)                                   kernel                 parallel unit
// computeActiveErrors + linearizeOplus          k_ba_edges             edge
// buildSystem: Hll, bl; Hpl (= Wb)            k_ba_points; k_ba_hpl  point (edges in CSR order); lead edge
// buildSystem: Hpp, bp                          k_ba_pose_chunk/final  256-edge chunk of one pose, then pose x entry
// setLambda + Dinv, Hpl Dinv, Hpl Dinv bl       k_ba_schur_points      point
// Hschur = Hpp - sum Hpl Dinv Hlp, bschur       k_ba_schur_gemm        (entry tile, point group); LDS-staged edges
//                                               k_ba_schur_reduce      entry (groups summed in fixed order)
// LinearSolverEigen on Hschur                   k_ba_dense_ldlt        one workgroup (LDS-resident up to order 112)
// xl = Dinv (bl - Hpl^T xp); update             k_ba_backsub, k_ba_update
//
// Deterministic: every sum has a fixed order (no floating-point atomics).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ba.h"
#include "device_math.h"

namespace deftri {
namespace dev {

#define TID (blockIdx.x * blockDim.x + threadIdx.x)

__device__ __forceinline__ void ba_huber(double delta, double e2, double &rho0, double &rho1) {
    // g2o RobustKernelHuber::robustify
    double dsqr = delta * delta;
    if (e2 <= dsqr) { rho0 = e2; rho1 = 1.0; }
    else { double se = sqrt(e2); rho0 = 2 * se * delta - dsqr; rho1 = delta / se; }
}

// e = obs - KB8(T_cw p) (g2oTypes.h:165-182); J_p = -Jpi R, J_T = -Jpi [-[X]x | I] (g2oTypes.cc:121-142)
__global__ void k_ba_edges(int E, const int32_t *__restrict__ ept, const int32_t *__restrict__ epose,
                           const double *__restrict__ obs, const double *__restrict__ info,
                           const uint8_t *__restrict__ robust, const uint8_t *__restrict__ active,
                           const uint8_t *__restrict__ sel, double hdelta,
                           const double *__restrict__ poses, const double *__restrict__ points,
                           const float *__restrict__ kb8, double *__restrict__ err, double *__restrict__ chi2raw,
                           double *__restrict__ chi, double *__restrict__ wgt, double *__restrict__ wr,
                           double *__restrict__ Jp, double *__restrict__ JT, int want_jac, int all_edges) {
    int e = TID;
    if (e >= E) return;
    const bool act = active[e] != 0;
    if (!all_edges) {
        if (!act) { chi[e] = 0.0; return; }
    } else if (sel && !sel[e]) {
        return;
    }
    const int k = epose[e];
    const double *pp = points + 3 * (int64_t)ept[e];
    const double p[3] = {pp[0], pp[1], pp[2]};
    SE3 T = se3_load(poses + 7 * k);
    double pc[3];
    se3_map(T, p, pc);
    const float pf[3] = {(float)pc[0], (float)pc[1], (float)pc[2]};
    float uv[2];
    kb8_project(kb8 + 8 * k, pf, uv);
    const double e0 = obs[2 * e] - (double)uv[0], e1 = obs[2 * e + 1] - (double)uv[1];
    const double om = info[e];
    const double c2 = e0 * (om * e0) + e1 * (om * e1);     // _error.dot(information() * _error)
    reinterpret_cast<double2 *>(err)[e] = double2{e0, e1};        // 16-B stores (per-edge records are 16-B aligned)
    chi2raw[e] = c2;
    double rho0 = c2, rho1 = 1.0;
    if (robust[e]) ba_huber(hdelta, c2, rho0, rho1);
    chi[e] = act ? rho0 : 0.0;
    if (!want_jac || !act) return;
    float jf[6];
    kb8_project_jac(kb8 + 8 * k, pf, jf);
    double A[6];
#pragma unroll
    for (int i = 0; i < 6; i++) A[i] = -(double)jf[i];
    double R[9];
    quat_to_mat(T.r, R);
    {
        double jp[6];
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int c = 0; c < 3; c++)
                jp[3 * r + c] = A[3 * r] * R[c] + A[3 * r + 1] * R[3 + c] + A[3 * r + 2] * R[6 + c];
        double2 *o2 = reinterpret_cast<double2 *>(Jp + 6 * (int64_t)e);
        o2[0] = double2{jp[0], jp[1]}; o2[1] = double2{jp[2], jp[3]}; o2[2] = double2{jp[4], jp[5]};
    }
    const double x = pc[0], y = pc[1], z = pc[2];
    // SE3deriv rows: [0 z -y 1 0 0; -z 0 x 0 1 0; y -x 0 0 0 1]
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const double a0 = A[3 * r], a1 = A[3 * r + 1], a2 = A[3 * r + 2];
        double2 *o2 = reinterpret_cast<double2 *>(JT + 12 * (int64_t)e + 6 * r);
        o2[0] = double2{a1 * (-z) + a2 * y, a0 * z + a2 * (-x)};
        o2[1] = double2{a0 * (-y) + a1 * x, a0};
        o2[2] = double2{a1, a2};
    }
    wgt[e] = rho1 * om;                                    // robustInformation = rho' * Omega
    reinterpret_cast<double2 *>(wr)[e] = double2{(-(om * e0)) * rho1, (-(om * e1)) * rho1};   // omega_r = -Omega e; *= rho'
}

// per point: Hll = sum J_p^T w J_p, bl = sum J_p^T omega_r, and the Hpl block of each (point, free
// pose) pair, Wb = sum J_T^T w J_p (6x3), stored at the pair's lead edge (duplicate observations of
// one point in one pose add into the same block, as g2o's Hpl)
__global__ void k_ba_points(int P, const int32_t *__restrict__ pt_ptr, const uint8_t *__restrict__ pt_free,
                            const uint8_t *__restrict__ active, const double *__restrict__ wgt,
                            const double *__restrict__ wr, const double *__restrict__ Jp, double *__restrict__ Hll,
                            double *__restrict__ bl) {
    int l = TID;
    if (l >= P || !pt_free[l]) return;
    double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, b[3] = {0, 0, 0};
    const int ebeg = pt_ptr[l], eend = pt_ptr[l + 1];
    for (int e = ebeg; e < eend; e++) {
        if (!active[e]) continue;
        const double w = wgt[e];
        const double *J = Jp + 6 * (int64_t)e;
        const double r0 = wr[2 * (int64_t)e], r1 = wr[2 * (int64_t)e + 1];
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const double a0 = J[c] * w, a1 = J[3 + c] * w;     // AtO(c, r)
#pragma unroll
            for (int d = 0; d < 3; d++) H[3 * c + d] += a0 * J[d] + a1 * J[3 + d];
            b[c] += J[c] * r0 + J[3 + c] * r1;
        }
    }
#pragma unroll
    for (int i = 0; i < 9; i++) Hll[9 * (int64_t)l + i] = H[i];
#pragma unroll
    for (int i = 0; i < 3; i++) bl[3 * (int64_t)l + i] = b[i];
}

// Hpl block of each (point, free pose) pair, one thread per lead edge (edge-parallel: coalesced
// J / JT reads and Wb writes).  The lead's own product (zero if the lead is inactive), then the
// active duplicate observations of the pair in edge order (g2o adds every edge's block).
__device__ __forceinline__ void ba_hpl_product(const double *J, const double *B, double w, double o[18], bool add) {
#pragma unroll
    for (int j = 0; j < 6; j++)
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const double v = (J[c] * w) * B[j] + (J[3 + c] * w) * B[6 + j];
            o[3 * j + c] = add ? o[3 * j + c] + v : v;
        }
}

__global__ void k_ba_hpl(int E, const int32_t *__restrict__ e_point, const int32_t *__restrict__ pt_ptr,
                         const uint8_t *__restrict__ pt_free, const uint8_t *__restrict__ active,
                         const int32_t *__restrict__ lead, const int32_t *__restrict__ pslot,
                         const double *__restrict__ wgt, const double *__restrict__ Jp,
                         const double *__restrict__ JT, double *__restrict__ Wb) {
    const int e = TID;
    if (e >= E || lead[e] != e || pslot[e] < 0) return;
    const int l = e_point[e];
    if (!pt_free[l]) return;
    double o[18];
    if (active[e]) ba_hpl_product(Jp + 6 * (int64_t)e, JT + 12 * (int64_t)e, wgt[e], o, false);
    else
#pragma unroll
        for (int i = 0; i < 18; i++) o[i] = 0.0;
    const int eend = pt_ptr[l + 1];
    for (int e2 = e + 1; e2 < eend; e2++)
        if (lead[e2] == e && active[e2]) ba_hpl_product(Jp + 6 * (int64_t)e2, JT + 12 * (int64_t)e2, wgt[e2], o, true);
#pragma unroll
    for (int i = 0; i < 18; i++) Wb[18 * (int64_t)e + i] = o[i];
}

// per-chunk partial sums of Hpp (36, full) and bp (6) of one free pose; 256 edges per chunk.
__global__ void __launch_bounds__(256) k_ba_pose_chunk(const int32_t *__restrict__ chunk_beg,
                                                       const int32_t *__restrict__ chunk_len,
                                                       const int32_t *__restrict__ pose_edges,
                                                       const uint8_t *__restrict__ active,
                                                       const double *__restrict__ wgt, const double *__restrict__ wr,
                                                       const double *__restrict__ JT, double *__restrict__ pchunk) {
    __shared__ double red[4][27];
    const int c = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    double v[27];
#pragma unroll
    for (int i = 0; i < 27; i++) v[i] = 0.0;
    if (t < chunk_len[c]) {
        const int e = pose_edges[chunk_beg[c] + t];
        if (active[e]) {
            const double w = wgt[e];
            const double *B = JT + 12 * (int64_t)e;
            const double r0 = wr[2 * (int64_t)e], r1 = wr[2 * (int64_t)e + 1];
            int q = 0;
#pragma unroll
            for (int i = 0; i < 6; i++) {
                const double a0 = B[i] * w, a1 = B[6 + i] * w;
#pragma unroll
                for (int j = 0; j <= i; j++) v[q++] = a0 * B[j] + a1 * B[6 + j];
            }
#pragma unroll
            for (int i = 0; i < 6; i++) v[21 + i] = B[i] * r0 + B[6 + i] * r1;
        }
    }
#pragma unroll
    for (int i = 0; i < 27; i++) {
        double x = v[i];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
        v[i] = x;
    }
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < 27; i++) red[wv][i] = v[i];
    __syncthreads();
    if (t < 27) {
        const double s = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
        pchunk[27 * (int64_t)c + t] = s;
    }
}

// Hpp (full 6x6) and bp per pose from its chunks in order; zeros for fixed / inactive poses
__global__ void __launch_bounds__(64) k_ba_pose_final(int K, const int32_t *__restrict__ pose_chunk_ptr,
                                                      const double *__restrict__ pchunk, double *__restrict__ Hpp,
                                                      double *__restrict__ bp) {
    const int id = blockIdx.x, lane = threadIdx.x;
    if (id >= K * 27) return;
    const int k = id / 27, q = id % 27;
    double s = 0.0;
    for (int c = pose_chunk_ptr[k] + lane; c < pose_chunk_ptr[k + 1]; c += 64) s += pchunk[27 * (int64_t)c + q];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane != 0) return;
    if (q < 21) {
        int i = 0;
        while ((i + 1) * (i + 2) / 2 <= q) i++;
        const int j = q - i * (i + 1) / 2;
        Hpp[36 * k + 6 * i + j] = s;
        Hpp[36 * k + 6 * j + i] = s;
    } else {
        bp[6 * k + (q - 21)] = s;
    }
}

__global__ void __launch_bounds__(256) k_ba_maxdiag(int P, int K, const uint8_t *__restrict__ pt_free,
                                                    const int32_t *__restrict__ pose_sidx,
                                                    const double *__restrict__ Hll, const double *__restrict__ Hpp,
                                                    double *__restrict__ part) {
    __shared__ double red[256];
    double mx = 0.0;
    const int n = P + K;
    const int chunk = (n + gridDim.x - 1) / gridDim.x;
    const int lo = blockIdx.x * chunk, hi = min(n, lo + chunk);
    for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        if (i < P) {
            if (!pt_free[i]) continue;
            const double *h = Hll + 9 * (int64_t)i;
            mx = fmax(mx, fmax(fabs(h[0]), fmax(fabs(h[4]), fabs(h[8]))));
        } else {
            const int k = i - P;
            if (pose_sidx[k] < 0) continue;
            for (int d = 0; d < 6; d++) mx = fmax(mx, fabs(Hpp[36 * k + 7 * d]));
        }
    }
    red[threadIdx.x] = mx;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + off]);
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void k_ba_max_final(int n, const double *__restrict__ part, double *__restrict__ out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double mx = 0.0;
        for (int i = 0; i < n; i++) mx = fmax(mx, part[i]);
        *out = mx;
    }
}

// setLambda on Hll; Dinv = (Hll + lambda I)^-1 (Eigen 3x3 cofactor inverse); db = Dinv bl;
// per edge with a free pose: Y = Wb Dinv (BDinv), v = Wb db
__global__ void k_ba_schur_points(int P, double lambda, const int32_t *__restrict__ pt_ptr,
                                  const uint8_t *__restrict__ pt_free, const int32_t *__restrict__ pslot,
                                  const double *__restrict__ Hll, const double *__restrict__ bl,
                                  const double *__restrict__ Wb, double *__restrict__ Dinv, double *__restrict__ Y,
                                  double *__restrict__ v, double *__restrict__ dbo, int want_v) {
    int l = TID;
    if (l >= P || !pt_free[l]) return;
    double m[9];
#pragma unroll
    for (int i = 0; i < 9; i++) m[i] = Hll[9 * (int64_t)l + i];
    m[0] += lambda; m[4] += lambda; m[8] += lambda;
#define M(i, j) m[3 * (i) + (j)]
#define COF(i, j) (M(((i) + 1) % 3, ((j) + 1) % 3) * M(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M(((i) + 1) % 3, ((j) + 2) % 3) * M(((i) + 2) % 3, ((j) + 1) % 3))
    const double c00 = COF(0, 0), c10 = COF(1, 0), c20 = COF(2, 0);
    const double det = (c00 * M(0, 0) + c10 * M(1, 0)) + c20 * M(2, 0);
    const double invdet = 1.0 / det;
    double Di[9];
    Di[0] = c00 * invdet; Di[1] = c10 * invdet; Di[2] = c20 * invdet;     // row 0 = cofactors_col0 * invdet
    Di[3] = COF(0, 1) * invdet; Di[4] = COF(1, 1) * invdet; Di[5] = COF(2, 1) * invdet;
    Di[6] = COF(0, 2) * invdet; Di[7] = COF(1, 2) * invdet; Di[8] = COF(2, 2) * invdet;
#undef COF
#undef M
#pragma unroll
    for (int i = 0; i < 9; i++) Dinv[9 * (int64_t)l + i] = Di[i];
    const double *b = bl + 3 * (int64_t)l;
    double db[3];
#pragma unroll
    for (int i = 0; i < 3; i++) db[i] = Di[3 * i] * b[0] + Di[3 * i + 1] * b[1] + Di[3 * i + 2] * b[2];
#pragma unroll
    for (int i = 0; i < 3; i++) dbo[3 * (int64_t)l + i] = db[i];
    if (!want_v) return;
    for (int e = pt_ptr[l]; e < pt_ptr[l + 1]; e++) {
        if (pslot[e] < 0) continue;
        const double *B = Wb + 18 * (int64_t)e;
        double *y = Y + 18 * (int64_t)e, *vv = v + 6 * (int64_t)e;
#pragma unroll
        for (int j = 0; j < 6; j++) {
#pragma unroll
            for (int c = 0; c < 3; c++)
                y[3 * j + c] = B[3 * j] * Di[c] + B[3 * j + 1] * Di[3 + c] + B[3 * j + 2] * Di[6 + c];
            vv[j] = B[3 * j] * db[0] + B[3 * j + 1] * db[1] + B[3 * j + 2] * db[2];
        }
    }
}

// Entries of the reduced system, enumerated as the lower triangle of S (row-major: (r, c), c <= r)
// followed by the ns rhs entries.  Workgroup (tile, group): 256 threads x kEpt entries of the
// tile, summed over the point stages of the group; the stage's edges (Y, Wb, v) and a
// (point, Schur block) -> edge table are staged in LDS.
constexpr int kEpt = 8;

__device__ __forceinline__ void tri_decode(int idx, int &r, int &c) {
    int rr = (int)((sqrt(8.0 * (double)idx + 1.0) - 1.0) * 0.5);
    while ((rr + 1) * (rr + 2) / 2 <= idx) rr++;
    while (rr * (rr + 1) / 2 > idx) rr--;
    r = rr;
    c = idx - rr * (rr + 1) / 2;
}

__global__ void __launch_bounds__(256) k_ba_schur_gemm(int ns, int nfree, const int32_t *__restrict__ group_stage,
                                                       const int32_t *__restrict__ stage_pt,
                                                       const int32_t *__restrict__ pt_ptr,
                                                       const int32_t *__restrict__ ept,
                                                       const int32_t *__restrict__ pslot,
                                                       const double *__restrict__ Y, const double *__restrict__ Wb,
                                                       const double *__restrict__ v, double *__restrict__ Spart) {
    extern __shared__ double lds[];
    double *sY = lds;                                    // [kBaStageEdges*18]
    double *sW = sY + kBaStageEdges * 18;                // [kBaStageEdges*18]
    double *sV = sW + kBaStageEdges * 18;                // [kBaStageEdges*6]
    int32_t *tab = (int32_t *)(sV + kBaStageEdges * 6);  // [kBaStageEdges * nfree]
    const int ntri = ns * (ns + 1) / 2, NE = ntri + ns;
    const int tile = blockIdx.x, g = blockIdx.y, t = threadIdx.x;
    int er[kEpt], ec[kEpt];
    double acc[kEpt];
#pragma unroll
    for (int q = 0; q < kEpt; q++) {
        const int idx = tile * 256 * kEpt + q * 256 + t;
        acc[q] = 0.0;
        if (idx >= NE) { er[q] = -1; ec[q] = -1; }
        else if (idx < ntri) tri_decode(idx, er[q], ec[q]);
        else { er[q] = idx - ntri; ec[q] = -1; }
    }
    for (int s = group_stage[g]; s < group_stage[g + 1]; s++) {
        const int p0 = stage_pt[s], p1 = stage_pt[s + 1];
        const int e0 = pt_ptr[p0], ne = pt_ptr[p1] - e0, np = p1 - p0;
        __syncthreads();
        for (int i = t; i < np * nfree; i += 256) tab[i] = -1;
        for (int i = t; i < ne * 18; i += 256) {
            sY[i] = Y[18 * (int64_t)e0 + i];
            sW[i] = Wb[18 * (int64_t)e0 + i];
        }
        for (int i = t; i < ne * 6; i += 256) sV[i] = v[6 * (int64_t)e0 + i];
        __syncthreads();
        for (int i = t; i < ne; i += 256) {
            const int sl = pslot[e0 + i];
            if (sl < 0) continue;
            tab[(ept[e0 + i] - p0) * nfree + sl] = i;      // edges are sorted by point
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kEpt; q++) {
            if (er[q] < 0) continue;
            const int a = er[q] / 6, ii = er[q] % 6;
            double sacc = 0.0;
            if (ec[q] >= 0) {
                const int b = ec[q] / 6, jj = ec[q] % 6;
                for (int lp = 0; lp < np; lp++) {
                    const int ea = tab[lp * nfree + a], eb = tab[lp * nfree + b];
                    if (ea < 0 || eb < 0) continue;
                    const double *y = sY + 18 * ea + 3 * ii, *w = sW + 18 * eb + 3 * jj;
                    sacc += y[0] * w[0] + y[1] * w[1] + y[2] * w[2];
                }
            } else {
                for (int lp = 0; lp < np; lp++) {
                    const int ea = tab[lp * nfree + a];
                    if (ea >= 0) sacc += sV[6 * ea + ii];
                }
            }
            acc[q] += sacc;
        }
    }
#pragma unroll
    for (int q = 0; q < kEpt; q++) {
        const int idx = tile * 256 * kEpt + q * 256 + t;
        if (idx < NE) Spart[(int64_t)g * NE + idx] = acc[q];
    }
}

// MFMA Schur complement: per 16-point stage, the stage's Hpl Dinv (Y) and Hpl (W) blocks are
// densified in LDS as k-major matrices Yd, Wd of npad rows (Schur dofs; row ns of Yd holds Dinv bl)
// and K = 48 columns (3 per point), then D += Yd Wd^T with v_mfma_f64_16x16x4 on the lower block
// triangle of 16x16 tiles.  D[i][j] (j <= i < ns) = sum Hpl_a Dinv Hlp_b; D[ns][j] = sum Hpl_b Dinv bl.
// One workgroup per group of consecutive stages (fixed order), partials reduced by k_ba_schur_reduce4.
typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int kMSP = 16;                 // points per MFMA stage

template <int NT>
__global__ void __launch_bounds__(256) k_ba_schur_mfma(int ns, int P, int stages_per_group,
                                                       const int32_t *__restrict__ pt_ptr,
                                                       const int32_t *__restrict__ ept,
                                                       const int32_t *__restrict__ pslot,
                                                       const uint8_t *__restrict__ pt_free,
                                                       const double *__restrict__ Dinv, const double *__restrict__ Wb,
                                                       const double *__restrict__ dbl, double *__restrict__ Spart) {
    constexpr int NP = 16 * NT, LDR = NP + 4, KD = 3 * kMSP;
    constexpr int NTILE = NT * (NT + 1) / 2, TPW = (NTILE + 3) / 4;
    __shared__ double Ys[KD * LDR], Ws[KD * LDR];
    const int g = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6, kl = lane >> 4, il = lane & 15;
    const int ntri = ns * (ns + 1) / 2, NE = ntri + ns;
    int tti[TPW], ttj[TPW];
    dbl4 acc[TPW];
#pragma unroll
    for (int q = 0; q < TPW; q++) {
        int idx = w + 4 * q;
        tti[q] = -1; ttj[q] = 0;
        if (idx < NTILE) {
            int i = 0;
            while ((i + 1) * (i + 2) / 2 <= idx) i++;
            tti[q] = i; ttj[q] = idx - i * (i + 1) / 2;
        }
        acc[q] = dbl4{0.0, 0.0, 0.0, 0.0};
    }
    const int nstage = (P + kMSP - 1) / kMSP;
    const int s0 = g * stages_per_group, s1 = min(nstage, s0 + stages_per_group);
    for (int s = s0; s < s1; s++) {
        const int p0 = s * kMSP, p1 = min(P, p0 + kMSP);
        const int e0 = pt_ptr[p0], e1 = pt_ptr[p1];
        __syncthreads();
        for (int i = t; i < KD * LDR; i += 256) { Ys[i] = 0.0; Ws[i] = 0.0; }
        __syncthreads();
        for (int i = t; i < (e1 - e0) * 18; i += 256) {
            const int e = e0 + i / 18, q = i % 18;
            const int sl = pslot[e];
            if (sl < 0) continue;
            const int l = ept[e], lp = l - p0, r = q / 3, c = q % 3;
            const double *wr = Wb + 18 * (int64_t)e + 3 * r, *di = Dinv + 9 * (int64_t)l + c;
            // Y = Hpl Dinv (BDinv of BlockSolver::solve), formed here instead of stored
            Ys[(3 * lp + c) * LDR + 6 * sl + r] = wr[0] * di[0] + wr[1] * di[3] + wr[2] * di[6];
            Ws[(3 * lp + c) * LDR + 6 * sl + r] = wr[c];
        }
        for (int i = t; i < (p1 - p0) * 3; i += 256) {
            const int lp = i / 3, c = i % 3, l = p0 + lp;
            Ys[(3 * lp + c) * LDR + ns] = pt_free[l] ? dbl[3 * (int64_t)l + c] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < TPW; q++) {
            if (tti[q] < 0) continue;
            const int ra = 16 * tti[q] + il, rb = 16 * ttj[q] + il;
#pragma unroll
            for (int kb = 0; kb < KD; kb += 4) {
                const double a = Ys[(kb + kl) * LDR + ra], b = Ws[(kb + kl) * LDR + rb];
                acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
            }
        }
    }
    double *out = Spart + (int64_t)g * NE;
#pragma unroll
    for (int q = 0; q < TPW; q++) {
        if (tti[q] < 0) continue;
#pragma unroll
        for (int gg = 0; gg < 4; gg++) {
            const int i = 16 * tti[q] + kl + 4 * gg, j = 16 * ttj[q] + il;
            if (i < ns && j <= i) out[i * (i + 1) / 2 + j] = acc[q][gg];
            else if (i == ns && j < ns) out[ntri + j] = acc[q][gg];
        }
    }
}

// Sred = -(sum over groups of the partials), groups in fixed order: 4 waves each sum a contiguous
// quarter of the groups for 64 entries, then the quarters are added in order
__global__ void __launch_bounds__(256) k_ba_schur_reduce4(int NE, int ngroup, const double *__restrict__ Spart,
                                                          double *__restrict__ Sred) {
    __shared__ double red[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int idx = blockIdx.x * 64 + lane;
    const int q = (ngroup + 3) / 4, g0 = w * q, g1 = min(ngroup, g0 + q);
    double s = 0.0;
    if (idx < NE)
        for (int g = g0; g < g1; g++) s += Spart[(int64_t)g * NE + idx];
    red[w][lane] = s;
    __syncthreads();
    if (w == 0 && idx < NE) Sred[idx] = -((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]));
}

__global__ void k_ba_schur_reduce(int NE, int ngroup, const double *__restrict__ Spart, double *__restrict__ Sred) {
    int idx = TID;
    if (idx >= NE) return;
    double s = 0.0;
    for (int g = 0; g < ngroup; g++) s += Spart[(int64_t)g * NE + idx];
    Sred[idx] = -s;
}

// S = Hpp + lambda I + Sred (lower triangle), rhs = bp + Sred_rhs; LDL^T (right-looking, no
// pivoting, as SimplicialLDLT); forward / diagonal / backward solve; xp -> dxp in pose order.
// flag: 1 if a pivot is zero (SimplicialLDLT NumericalIssue) or, with dense_positive, negative
// (LinearSolverDense: Eigen LDLT::isPositive).
template <bool kLds>
__global__ void __launch_bounds__(1024) k_ba_dense_ldlt(int ns, int K, double lambda, int dense_positive,
                                                        const int32_t *__restrict__ pose_sidx,
                                                        const double *__restrict__ Hpp,
                                                        const double *__restrict__ bp,
                                                        const double *__restrict__ Sred, double *__restrict__ Sg,
                                                        double *__restrict__ xp, double *__restrict__ dxp,
                                                        int *__restrict__ flag) {
    extern __shared__ double lds[];
    double *A = kLds ? lds : Sg;                          // ns x ns row-major, lower triangle used
    __shared__ double x[1200 + 8];
    __shared__ int s_pose[200];
    __shared__ int bad;
    const int t = threadIdx.x, nt = blockDim.x;
    const int ntri = ns * (ns + 1) / 2;
    if (t == 0) bad = 0;
    for (int k = t; k < K; k += nt) if (pose_sidx[k] >= 0) s_pose[pose_sidx[k]] = k;
    __syncthreads();
    for (int idx = t; idx < ntri; idx += nt) {
        int r, c;
        tri_decode(idx, r, c);
        const int a = r / 6, b = c / 6;
        double h = Sred[idx];
        if (a == b) h = Hpp[36 * s_pose[a] + 6 * (r % 6) + (c % 6)] + h;
        if (r == c) h = (Hpp[36 * s_pose[a] + 7 * (r % 6)] + lambda) + Sred[idx];
        A[(int64_t)r * ns + c] = h;
    }
    for (int r = t; r < ns; r += nt) x[r] = bp[6 * s_pose[r / 6] + r % 6] + Sred[ntri + r];
    __syncthreads();
    // right-looking LDL^T: step k updates the trailing lower triangle with the unscaled column k
    // and scales column k-1 (no longer read)
    for (int k = 0; k < ns; k++) {
        const double d = A[(int64_t)k * ns + k];
        if (t == 0 && (d == 0.0 || (dense_positive && d < 0.0))) bad = 1;
        const double dinv = 1.0 / d;
        const int m = ns - k - 1;
        const int nupd = m * (m + 1) / 2;
        for (int u = t; u < nupd; u += nt) {
            int i, j;
            tri_decode(u, i, j);
            i += k + 1; j += k + 1;
            A[(int64_t)i * ns + j] -= A[(int64_t)i * ns + k] * (A[(int64_t)j * ns + k] * dinv);
        }
        if (k > 0) {
            const double dp = 1.0 / A[(int64_t)(k - 1) * ns + (k - 1)];
            for (int i = k + t; i < ns; i += nt) A[(int64_t)i * ns + (k - 1)] *= dp;
        }
        __syncthreads();
    }
    // forward L y = rhs
    for (int k = 0; k < ns; k++) {
        const double yk = x[k];
        for (int i = k + 1 + t; i < ns; i += nt) x[i] -= A[(int64_t)i * ns + k] * yk;
        __syncthreads();
    }
    for (int i = t; i < ns; i += nt) x[i] = x[i] / A[(int64_t)i * ns + i];
    __syncthreads();
    // backward L^T x = z
    for (int k = ns - 1; k >= 0; k--) {
        const double xk = x[k];
        for (int i = t; i < k; i += nt) x[i] -= A[(int64_t)k * ns + i] * xk;
        __syncthreads();
    }
    for (int r = t; r < ns; r += nt) xp[r] = x[r];
    for (int id = t; id < 6 * K; id += nt) {
        const int sl = pose_sidx[id / 6];
        dxp[id] = sl >= 0 ? x[6 * sl + id % 6] : 0.0;
    }
    if (t == 0 && bad) *flag = 1;
}

// xl = Dinv (bl - Hpl^T xp)  (BlockSolver: cl = bl; cl += Hpl^T (-xp); xl = Dinv cl)
__global__ void k_ba_backsub(int P, const int32_t *__restrict__ pt_ptr, const uint8_t *__restrict__ pt_free,
                             const int32_t *__restrict__ pslot, const double *__restrict__ Wb,
                             const double *__restrict__ Dinv, const double *__restrict__ bl,
                             const double *__restrict__ xp, double *__restrict__ dxl) {
    int l = TID;
    if (l >= P || !pt_free[l]) return;
    double c[3] = {bl[3 * (int64_t)l], bl[3 * (int64_t)l + 1], bl[3 * (int64_t)l + 2]};
    for (int e = pt_ptr[l]; e < pt_ptr[l + 1]; e++) {
        const int sl = pslot[e];
        if (sl < 0) continue;
        const double *B = Wb + 18 * (int64_t)e;
        const double *xx = xp + 6 * sl;
#pragma unroll
        for (int cc = 0; cc < 3; cc++) {
            double s = 0.0;
#pragma unroll
            for (int j = 0; j < 6; j++) s += B[3 * j + cc] * (-xx[j]);
            c[cc] += s;
        }
    }
    const double *D = Dinv + 9 * (int64_t)l;
#pragma unroll
    for (int i = 0; i < 3; i++) dxl[3 * (int64_t)l + i] = D[3 * i] * c[0] + D[3 * i + 1] * c[1] + D[3 * i + 2] * c[2];
}

// VertexSE3Expmap::oplusImpl (T <- exp(d) T) for free poses; VertexSBAPointXYZ += d for free points
__global__ void k_ba_update(int P, int K, const uint8_t *__restrict__ pt_free, const int32_t *__restrict__ pose_sidx,
                           const double *__restrict__ dxl, const double *__restrict__ dxp,
                           double *__restrict__ points, double *__restrict__ poses) {
    int i = TID;
    if (i < P && pt_free[i]) {
#pragma unroll
        for (int k = 0; k < 3; k++) points[3 * (int64_t)i + k] += dxl[3 * (int64_t)i + k];
    }
    if (i < K && pose_sidx[i] >= 0) {
        double u[6];
        for (int k = 0; k < 6; k++) u[k] = dxp[6 * i + k];
        SE3 T = se3_load(poses + 7 * i);
        SE3 Ex = se3_exp(u);
        se3_store(se3_mul(Ex, T), poses + 7 * i);
    }
}

// per edge (caller order via perm): cached chi2 and isDepthPositive at the current state
__global__ void k_ba_edge_query(int E, const int32_t *__restrict__ perm, const int32_t *__restrict__ ept,
                                const int32_t *__restrict__ epose, const double *__restrict__ poses,
                                const double *__restrict__ points, const double *__restrict__ chi2raw,
                                double *__restrict__ chi2_out, uint8_t *__restrict__ dpos_out) {
    int e = TID;
    if (e >= E) return;
    const int o = perm[e];
    if (chi2_out) chi2_out[o] = chi2raw[e];
    if (dpos_out) {
        const double *pp = points + 3 * (int64_t)ept[e];
        const double p[3] = {pp[0], pp[1], pp[2]};
        SE3 T = se3_load(poses + 7 * epose[e]);
        double pc[3];
        se3_map(T, p, pc);
        dpos_out[o] = pc[2] > 0.0 ? 1 : 0;
    }
}

}  // namespace dev

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
static thread_local KProf *g_baprof = nullptr;
void ba_set_profiler(KProf *p) { g_baprof = p; }
static hipEvent_t ba_prof_event() {
    KProf &P = *g_baprof;
    if (P.next == P.pool.size()) { hipEvent_t e; hipEventCreate(&e); P.pool.push_back(e); }
    return P.pool[P.next++];
}
#define BALAUNCH(NAME, KER, GRID, BLOCK, SHM, ST, ...)                              \
    do {                                                                             \
        if (dim3(GRID).x == 0) break;                  /* (n = 0: not launched) */   \
        hipEvent_t e0_ = nullptr;                                                    \
        if (g_baprof) { e0_ = ba_prof_event(); hipEventRecord(e0_, ST); }            \
        hipLaunchKernelGGL(KER, GRID, BLOCK, SHM, ST, __VA_ARGS__);                  \
        if (g_baprof) {                                                              \
            hipEvent_t e1_ = ba_prof_event();                                        \
            hipEventRecord(e1_, ST);                                                 \
            g_baprof->recs.push_back({NAME, e0_, e1_, dim3(GRID).x, 0.0, -1});       \
        }                                                                            \
    } while (0)

static inline unsigned nbk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

void ba_launch_edges(const BADev &B, hipStream_t st, bool want_jac, bool all_edges, const uint8_t *sel) {
    if (B.E <= 0) return;
    BALAUNCH("ba_edges", dev::k_ba_edges, dim3(nbk(B.E, 128)), dim3(128), 0, st, B.E, B.e_point, B.e_pose, B.obs,
             B.info, B.robust, B.active, sel, B.huber, B.poses, B.points, B.kb8, B.err, B.chi2raw, B.chi, B.wgt,
             B.wr, B.Jp, B.JT, want_jac ? 1 : 0, all_edges ? 1 : 0);
}

namespace dev {
// initializeOptimization(level) (g2o; reference g2oBundleAdjustment.cc:56-60 / 297-305): an edge
// is active at `level` unless both its vertices are fixed; a pose / point is active when one of its
// edges is.  Flags are set with plain stores of 1 (idempotent: the result has no order).
__global__ void k_ba_active(int E, int level, const uint8_t *__restrict__ e_level, const int32_t *__restrict__ e_point,
                            const int32_t *__restrict__ e_pose, const uint8_t *__restrict__ pt_fixed,
                            const uint8_t *__restrict__ pose_fixed, uint8_t *__restrict__ active,
                            int32_t *__restrict__ pose_flag, uint8_t *__restrict__ pt_act) {
    const int s = TID;
    if (s >= E) return;
    const int l = e_point[s], k = e_pose[s];
    const bool a = e_level[s] == level && !(pt_fixed[l] && pose_fixed[k]);
    active[s] = a ? 1 : 0;
    if (a) { pose_flag[k] = 1; pt_act[l] = 1; }
}

__global__ void k_ba_free_points(int P, const uint8_t *__restrict__ pt_act, const uint8_t *__restrict__ pt_fixed,
                                 uint8_t *__restrict__ pt_free, int32_t *__restrict__ count) {
    const int l = TID;
    if (l >= P) return;
    const bool f = pt_act[l] && !pt_fixed[l];
    pt_free[l] = f ? 1 : 0;
    if (f) atomicAdd(count, 1);                       // integer count: order-independent
}

// Schur slot on the lead edge of each (point, pose) pair with an active edge, free point and free
// pose (every such edge of the pair writes the same value)
__global__ void k_ba_pslot(int E, const uint8_t *__restrict__ active, const int32_t *__restrict__ e_point,
                           const int32_t *__restrict__ e_pose, const uint8_t *__restrict__ pt_free,
                           const int32_t *__restrict__ pose_sidx, const int32_t *__restrict__ lead,
                           int32_t *__restrict__ pslot) {
    const int s = TID;
    if (s >= E || !active[s]) return;
    const int l = e_point[s], k = e_pose[s];
    if (pt_free[l] && pose_sidx[k] >= 0) pslot[lead[s]] = pose_sidx[k];
}
}  // namespace dev

void ba_launch_active(const BADev &B, int level, hipStream_t st) {
    hipMemsetAsync(B.pose_flag, 0, sizeof(int32_t) * (size_t)std::max(B.K, 1), st);
    hipMemsetAsync(B.pt_act, 0, (size_t)std::max(B.P, 1), st);
    if (B.E > 0)
        BALAUNCH("ba_active", dev::k_ba_active, dim3(nbk(B.E, 256)), dim3(256), 0, st, B.E, level, B.e_level,
                 B.e_point, B.e_pose, B.pt_fixed, B.pose_fixed, B.active, B.pose_flag, B.pt_act);
}

void ba_launch_free_slots(const BADev &B, hipStream_t st) {
    hipMemsetAsync(B.icount, 0, sizeof(int32_t), st);
    hipMemsetAsync(B.pslot, 0xFF, sizeof(int32_t) * (size_t)std::max(B.E, 1), st);     // -1
    if (B.P > 0)
        BALAUNCH("ba_free_points", dev::k_ba_free_points, dim3(nbk(B.P, 256)), dim3(256), 0, st, B.P, B.pt_act,
                 B.pt_fixed, B.pt_free, B.icount);
    if (B.E > 0)
        BALAUNCH("ba_pslot", dev::k_ba_pslot, dim3(nbk(B.E, 256)), dim3(256), 0, st, B.E, B.active, B.e_point,
                 B.e_pose, B.pt_free, B.pose_sidx, B.lead, B.pslot);
}

void ba_launch_chi2_sum(const BADev &B, double *out, hipStream_t st) {
    launch_sum(B.E, B.chi, nullptr, 0, 0, B.part, 256, out, st);
}

void ba_launch_points(const BADev &B, hipStream_t st) {
    if (B.P <= 0) return;
    BALAUNCH("ba_points", dev::k_ba_points, dim3(nbk(B.P, 128)), dim3(128), 0, st, B.P, B.pt_ptr, B.pt_free,
             B.active, B.wgt, B.wr, B.Jp, B.Hll, B.bl);
    if (B.E > 0)
        BALAUNCH("ba_hpl", dev::k_ba_hpl, dim3(nbk(B.E, 256)), dim3(256), 0, st, B.E, B.e_point, B.pt_ptr, B.pt_free,
                 B.active, B.lead, B.pslot, B.wgt, B.Jp, B.JT, B.Wb);
}

void ba_launch_poses(const BADev &B, hipStream_t st) {
    hipMemsetAsync(B.Hpp, 0, sizeof(double) * 42 * (size_t)B.K, st);
    if (B.nchunk > 0)
        BALAUNCH("ba_pose_chunk", dev::k_ba_pose_chunk, dim3(B.nchunk), dim3(256), 0, st, B.chunk_beg, B.chunk_len,
                 B.pose_edges, B.active, B.wgt, B.wr, B.JT, B.pchunk);
    if (B.K > 0)
        BALAUNCH("ba_pose_final", dev::k_ba_pose_final, dim3(27 * B.K), dim3(64), 0, st, B.K,
                 B.pose_chunk_ptr, B.pchunk, B.Hpp, B.bp);
}

void ba_launch_maxdiag(const BADev &B, double *out, hipStream_t st) {
    BALAUNCH("ba_maxdiag", dev::k_ba_maxdiag, dim3(64), dim3(256), 0, st, B.P, B.K, B.pt_free, B.pose_sidx, B.Hll,
             B.Hpp, B.part);
    BALAUNCH("ba_max_final", dev::k_ba_max_final, dim3(1), dim3(64), 0, st, 64, B.part, out);
}

static size_t schur_lds(int nfree) {
    return sizeof(double) * (size_t)kBaStageEdges * (18 + 18 + 6) + sizeof(int32_t) * (size_t)kBaStageEdges * nfree;
}

void ba_launch_schur(const BADev &B, double lambda, hipStream_t st) {
    if (B.P > 0)
        BALAUNCH("ba_schur_points", dev::k_ba_schur_points, dim3(nbk(B.P, 128)), dim3(128), 0, st, B.P, lambda,
                 B.pt_ptr, B.pt_free, B.pslot, B.Hll, B.bl, B.Wb, B.Dinv, B.Y, B.v, B.dbl,
                 (B.mgroup > 0 && B.ns < 128) ? 0 : 1);
    const int NE = B.ns * (B.ns + 1) / 2 + B.ns;
    if (B.ns == 0) return;
    if (B.mgroup > 0 && B.ns < 128) {                   // MFMA path (npad = 16 NT > ns)
        const int nt = B.ns / 16 + 1;
#define MF(NTV)                                                                                         \
        BALAUNCH("ba_schur_mfma", dev::k_ba_schur_mfma<NTV>, dim3(B.mgroup), dim3(256), 0, st, B.ns, B.P,   \
                 B.mstages_per_group, B.pt_ptr, B.e_point, B.pslot, B.pt_free, B.Dinv, B.Wb, B.dbl, B.Spart)
        switch (nt) {
            case 1: MF(1); break;
            case 2: MF(2); break;
            case 3: MF(3); break;
            case 4: MF(4); break;
            case 5: MF(5); break;
            case 6: MF(6); break;
            case 7: MF(7); break;
            default: MF(8); break;
        }
#undef MF
        BALAUNCH("ba_schur_reduce", dev::k_ba_schur_reduce4, dim3(nbk(NE, 64)), dim3(256), 0, st, NE, B.mgroup,
                 B.Spart, B.Sred);
    } else if (B.ngroup > 0) {
        const int ntile = (NE + 256 * dev::kEpt - 1) / (256 * dev::kEpt);
        static bool attr = false;
        if (!attr) {
            hipFuncSetAttribute((const void *)dev::k_ba_schur_gemm, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)schur_lds(200));
            attr = true;
        }
        BALAUNCH("ba_schur_gemm", dev::k_ba_schur_gemm, dim3(ntile, B.ngroup), dim3(256), schur_lds(B.nfree), st,
                 B.ns, B.nfree, B.group_stage, B.stage_pt, B.pt_ptr, B.e_point, B.pslot, B.Y, B.Wb, B.v, B.Spart);
        BALAUNCH("ba_schur_reduce", dev::k_ba_schur_reduce, dim3(nbk(NE, 256)), dim3(256), 0, st, NE, B.ngroup,
                 B.Spart, B.Sred);
    } else {
        hipMemsetAsync(B.Sred, 0, sizeof(double) * (size_t)NE, st);
    }
}

void ba_launch_dense_solve(const BADev &B, double lambda, hipStream_t st) {
    const int dense_positive = B.dense_positive;
    if (B.ns == 0) { hipMemsetAsync(B.dxp, 0, sizeof(double) * 6 * (size_t)B.K, st); return; }
    const int threads = B.ns <= 32 ? 256 : 1024;
    if (B.ns <= kBaLdsMaxN) {
        static bool attr = false;
        if (!attr) {
            hipFuncSetAttribute((const void *)dev::k_ba_dense_ldlt<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)(sizeof(double) * kBaLdsMaxN * kBaLdsMaxN));
            attr = true;
        }
        BALAUNCH("ba_dense_ldlt", dev::k_ba_dense_ldlt<true>, dim3(1), dim3(threads),
                 sizeof(double) * (size_t)B.ns * B.ns, st, B.ns, B.K, lambda, dense_positive, B.pose_sidx, B.Hpp,
                 B.bp, B.Sred, B.S, B.xp, B.dxp, B.flag);
    } else
        BALAUNCH("ba_dense_ldlt", dev::k_ba_dense_ldlt<false>, dim3(1), dim3(threads), 0, st, B.ns, B.K, lambda,
                 dense_positive, B.pose_sidx, B.Hpp, B.bp, B.Sred, B.S, B.xp, B.dxp, B.flag);
}

void ba_launch_backsub_update(const BADev &B, hipStream_t st) {
    if (B.P > 0)
        BALAUNCH("ba_backsub", dev::k_ba_backsub, dim3(nbk(B.P, 128)), dim3(128), 0, st, B.P, B.pt_ptr, B.pt_free,
                 B.pslot, B.Wb, B.Dinv, B.bl, B.xp, B.dxl);
    const int n = B.P > B.K ? B.P : B.K;
    if (n > 0)
        BALAUNCH("ba_update", dev::k_ba_update, dim3(nbk(n, 128)), dim3(128), 0, st, B.P, B.K, B.pt_free,
                 B.pose_sidx, B.dxl, B.dxp, B.points, B.poses);
}

void ba_launch_scale(const BADev &B, double lambda, double *out_pts, double *out_pose, hipStream_t st) {
    launch_sum(3 * (int64_t)B.P, B.dxl, B.bl, lambda, 1, B.part, 256, out_pts, st);
    launch_sum(6 * (int64_t)B.K, B.dxp, B.bp, lambda, 1, B.part + 256, 1, out_pose, st);
}

void ba_launch_edge_chi2(const BADev &B, const int32_t *perm, double *chi2_out, uint8_t *dpos_out, hipStream_t st) {
    if (B.E <= 0) return;
    BALAUNCH("ba_edge_query", dev::k_ba_edge_query, dim3(nbk(B.E, 128)), dim3(128), 0, st, B.E, perm, B.e_point,
             B.e_pose, B.poses, B.points, B.chi2raw, chi2_out, dpos_out);
}

}  // namespace deftri
