// spcg.hip — gfx950 kernels of the point-sharded matrix-free PCG plan (spcg.h).
//
// Replaces (reference / g2o): buildSystem + the linear solve of OptimizationAlgorithmLevenberg::solve
// (BlockSolverX + LinearSolverEigen SimplicialLDLT, built at g2oBundleAdjustment.cc:619-628, run by
// optimize() at :959-962) with block-Jacobi PCG on an operator that is never assembled.
//
// Per LM iteration (after the edges are linearized, kernels.hip k_lin_*):
//   k_sp_glin_rows    own rows: the row's 3x3 diagonal block of H (incidences + folded single-point
//                     edges), D_v (its reprojection / depth part), b_v, c_e = W J_p J_s per depth edge
//   k_sp_glin_blocks  per phase-1 block: the heavy vertices' H / b partials (owned edges only)
//   k_sp_glin_heavy   heavy H / b from the block partials (rank sums; all-reduced by the host)
// Per CG iteration it (sharded: 6 launches, two all-reduces and the halo exchange of the boundary
// rows' (z, p); one rank, merged chain (default): 2 launches — phase 1 also forms p.Ap and alpha,
// phase 2 also the update and the next (r.z, r.r); one rank, DEFTRI_SP_NO_MERGE=1: 3 launches —
// k_sp_dots runs in the last workgroup of the update before it (or of the setup), and k_sp_heavy in
// the last workgroup of k_sp_phase2 when the heavy vertices have few block partials (G.fuse_heavy)):
//   k_sp_dots    (r.z, r.r) from the previous update's row-block partials
//   k_sp_phase1  per local ARAP edge s_e = W_e J_e p, per block J_T^T s (T_g) / depth-scale sums
//   k_sp_phase2  per own row q_v (p formed from (z, p_prev) on the fly and stored), partial p.q
//   k_sp_heavy   heavy q from the block partials, p.q, alpha (breakdown -> status)
//   k_sp_update  x += alpha p, r -= alpha q, z = M r, partial (r.z, r.r)
// Each kernel first tests the iteration's state from the reduced scalars (converged: ||r||^2 <=
// tol^2 ||b||^2 on the recurrence residual; budget; breakdown) and returns at once past the end, so
// the host may queue more iterations than a solve needs.  No atomics; fixed-order sums.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <type_traits>

#include "spcg.h"
#include "ticket.h"
#include "wave.h"

namespace deftri {
namespace sp {

using wv::wave_sum;
using wv::wave_max;

// fixed-order sum of a 256-thread workgroup: wave butterflies, then (w0 + w1) + (w2 + w3)
__device__ __forceinline__ double block_sum(double v, double *red4) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    v = wave_sum(v);
    if (lane == 0) red4[w] = v;
    __syncthreads();
    const double s = (red4[0] + red4[1]) + (red4[2] + red4[3]);
    __syncthreads();
    return s;
}

__device__ __forceinline__ double pval(const double2 *__restrict__ zp, double beta, int64_t i) {
    const double2 v = zp[i];
    return __fma_rn(beta, v.y, v.x);
}

// the state of CG iteration `it`: 0 run it (beta set); otherwise the status that stops it — the one
// already recorded (rec[0]: breakdown, bad block, converged earlier), a stop the merged chain's
// phase 2 left for this iteration (red[it][2]: breakdown, hand-off timeout), kSpConverged or
// kSpBudget.  Every input is fixed for the whole launch except rec[0], which a launch writes only
// when every one of its workgroups stops, so all workgroups of a launch take the same branch
__device__ __forceinline__ int it_state(const SpDev &G, int it, double &beta) {
    beta = 0.0;
    if (G.rec[0] != 0.0) return (int)G.rec[0];
    const double *rk = G.red + (int64_t)kSpRed * it;
    if (rk[2] != 0.0) return (int)rk[2];
    if (rk[1] <= G.tol2 * G.red[1]) return kSpConverged;
    if (it >= G.max_it) return kSpBudget;
    if (it > 0) beta = rk[0] / G.red[(int64_t)kSpRed * (it - 1)];
    return 0;
}

// record the status that stopped iteration it (one thread; the first stop wins)
__device__ __forceinline__ void record_stop(const SpDev &G, int it, int st) {
    if (G.rec[0] == 0.0) {
        G.rec[0] = st;
        G.rec[1] = it;
    }
}

// XCD-aware row blocks: workgroup b runs on XCD b % 8; the launch has 8 ceil(nrb / 8) row
// workgroups and workgroup b takes logical row block (b % 8) seg + b / 8 (seg = ceil(nrb / 8)), so
// each XCD walks one contiguous run of rows (its neighbours' s_e / p stay in that XCD's L2).
// Logical blocks >= nrb are empty (they still take part in the launch's hand-off).
__host__ __device__ __forceinline__ int row_grid(int nrb) { return 8 * ((max(nrb, 1) + 7) / 8); }
__device__ __forceinline__ int row_block(int b, int nrb) {
    const int seg = (max(nrb, 1) + 7) / 8;
    return (b & 7) * seg + (b >> 3);
}

__device__ __forceinline__ int heavy_dof(const SpDev &G, int h) { return h < G.Q ? 6 * h : 6 * G.Q + (h - G.Q); }

// device-driven LM: the slot's gate words (spcg.h SpDev::gate / lgate) and its lambda
__device__ __forceinline__ bool gated_off(const int *g) { return g && !*g; }
__device__ __forceinline__ double lam_of(const SpDev &G, double lam) { return G.lam_dev ? *G.lam_dev : lam; }

// Last-workgroup hand-off (G.fuse).  A workgroup's partials are published by thread 0 with
// agent-scope relaxed atomic stores (coherent across the XCDs' L2s, no L2 write-back); after its
// stores are acknowledged (s_waitcnt) it takes a ticket; the workgroup that draws the last ticket
// reads every partial with agent-scope atomic loads and forms the sums in a fixed order, so the
// result does not depend on the arrival order.  (Plain stores and loads around __threadfence()
// instead: a whole-L2 write-back per workgroup on gfx950, measured slower in round 3.)
__device__ __forceinline__ void publish(double *p, double v) { st_sc1(p, v); }
__device__ __forceinline__ double fetch(const double *p) {     // a partial published in this launch
    return ld_sc1(p);
}

// ---- per LM iteration -----------------------------------------------------------------------------
__device__ __forceinline__ int tri3(int a, int b) { return a * (a + 1) / 2 + b; }   // a >= b
__device__ __forceinline__ int tri6(int a, int b) { return a * (a + 1) / 2 + b; }

// own rows in the phase-2 wave layout (one lane per row, 64 rows per wave): the row's 3x3 diagonal
// block of H (reprojection and depth folded into D_v, then the ARAP incidences), b_v, the depth
// couplings c_e = W J_p J_s; and, slot by slot, the packed J slices phase 2 reads (an ARAP slice is
// gathered once: added into H_v and stored).  Slots of a row: its incidences in the plan's order,
// then its depth couplings, then padding.
// GU (G.glu): slots per step — 8 (3 waves per SIMD) or 4 (5 waves per SIMD: a C2-size grid of
// ~3100 waves then fits the chip in one round)
template <class JT, int GU>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GU == 4 ? 5 : GU == 6 ? 4 : 1, GU == 4 ? 5 : GU == 6 ? 4 : 3)))
k_sp_glin_rows(const SpDev G, JT *__restrict__ pj) {
    __shared__ double red4[4];
    if (gated_off(G.lgate)) return;
    const int lb = row_block(blockIdx.x, G.nrb2);
    const int w = lb * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    double mx = 0.0;
    if (w < G.nwaves) {
        const int l = G.rowmap[64 * w + lane];
        double D[6] = {0, 0, 0, 0, 0, 0}, bb[3] = {0, 0, 0};
        if (l >= 0) {
            for (int j = G.rep_off[l]; j < G.rep_off[l + 1]; j++) {     // reprojection: 2 x 3, W scalar
                const double *J = G.Jr + 6 * (int64_t)j;
                const double wt = G.Wr[j];
#pragma unroll
                for (int r = 0; r < 2; r++) {
                    const double er = G.Er[2 * (int64_t)j + r];
#pragma unroll
                    for (int a = 0; a < 3; a++) {
                        const double ja = J[3 * r + a] * wt;
#pragma unroll
                        for (int c = 0; c <= a; c++) D[tri3(a, c)] += ja * J[3 * r + c];
                        bb[a] -= J[3 * r + a] * (wt * er);
                    }
                }
            }
            // depth: J_p (3), J_s — four edges' loads issued before the first is used (several pairs:
            // a row has one per pair), the sums in edge order
            const int d0 = G.dep_off[l], d1 = G.dep_off[l + 1];
            for (int jb = d0; jb < d1; jb += 4) {
                double Jb[4][4], wb[4], eb[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int64_t j = jb + u < d1 ? jb + u : jb;
#pragma unroll
                    for (int c = 0; c < 4; c++) Jb[u][c] = G.Jd[4 * j + c];
                    wb[u] = G.Wd[j];
                    eb[u] = G.Ed[j];
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (jb + u >= d1) break;
                    const int64_t j = jb + u;
                    const double *J = Jb[u];
                    const double wt = wb[u], er = eb[u];
#pragma unroll
                    for (int a = 0; a < 3; a++) {
                        const double ja = J[a] * wt;
#pragma unroll
                        for (int c = 0; c <= a; c++) D[tri3(a, c)] += ja * J[c];
                        bb[a] -= J[a] * (wt * er);
                        G.cdep[3 * j + a] = ja * J[3];
                    }
                    G.wss[j] = (J[3] * wt) * J[3];
                }
            }
        }
        double H[6];
#pragma unroll
        for (int k = 0; k < 6; k++) H[k] = D[k];
        const int64_t n = G.nslots * 64;
        // one slot: its J slice (ARAP incidence le << 2 | role, or the depth coupling of the row's
        // edge -2 - m), weight and error (ARAP) / J_s (depth).  load(): the same five loads on every
        // path (selected addresses; padding reads ARAP edge 0); value(): selects only — so the four
        // slots of a step issue all their loads before the first is used
        struct Raw { double j0, j1, j2, w, x; };
        const double *__restrict__ Ja = G.Ja, *__restrict__ Wa = G.Wa, *__restrict__ Ea = G.Ea;
        const double *__restrict__ Jd = G.Jd, *__restrict__ Wd = G.Wd;
        const int64_t jld = G.jld;
        // one pair: every ARAP edge's W is the pair's Omega (k_lin_arap stores W = pinfo[pair]), one
        // uniform load instead of a gather per slot
        const bool w1 = G.Q == 1 && G.pinfo != nullptr;
        auto load = [&](int m) -> Raw {
            const bool dep = m <= -2;
            const int mm = max(m, 0), jj = max(-2 - m, 0);
            const double *pa = Ja + (int64_t)(3 * (mm & 3)) * jld + (mm >> 2);   // ARAP (padding: edge 0)
            const double *pd = Jd + 4 * (int64_t)jj;
            const double *Jc = dep ? pd : pa;
            const int64_t st = dep ? 1 : jld;
            const double *W = dep ? Wd + jj : w1 ? G.pinfo : Wa + (mm >> 2);
            const double *X = dep ? pd + 3 : Ea + (mm >> 2);
            return Raw{Jc[0], Jc[st], Jc[2 * st], *W, *X};
        };
        auto value = [&](int m, const Raw &r, double *v, double &wt, double &er) {
            const bool arap = m >= 0, dep = m <= -2;
            v[0] = dep ? (r.j0 * r.w) * r.x : arap ? r.j0 : 0.0;
            v[1] = dep ? (r.j1 * r.w) * r.x : arap ? r.j1 : 0.0;
            v[2] = dep ? (r.j2 * r.w) * r.x : arap ? r.j2 : 0.0;
            wt = arap ? r.w : 0.0;
            er = arap ? r.x : 0.0;
        };
        // branch-free: depth couplings and padding come with wt = er = 0 from value() and add exact
        // zeros (a per-slot branch here made the compiler serialize the slots' loads)
        auto add = [&](const double *v, double wt, double er) {
#pragma unroll
            for (int a = 0; a < 3; a++) {
                const double ja = v[a] * wt;
#pragma unroll
                for (int c = 0; c <= a; c++) H[tri3(a, c)] += ja * v[c];
                bb[a] -= v[a] * (wt * er);
            }
        };
        // U slots per step: indices, loads, then in order.  A clamped step (the last, fewer than U
        // slots left; the count is uniform in the wave) repeats the last slot in place of the missing
        // ones with wt = er = 0 (exact zeros added; its slice stored again, the same value)
        int64_t k = G.woff[w] * 64 + lane;
        const int64_t k1 = G.woff[w + 1] * 64 + lane;
        auto step = [&](auto U_, bool clamp) {
            constexpr int U = decltype(U_)::value;
            int m[U];
            int64_t kk[U];
            bool in[U];
            Raw r[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                in[u] = !clamp || k + 64 * u < k1;
                kk[u] = in[u] ? k + 64 * u : k1 - 64;
            }
#pragma unroll
            for (int u = 0; u < U; u++) m[u] = G.pmap[kk[u]];
#pragma unroll
            for (int u = 0; u < U; u++) r[u] = load(m[u]);
#pragma unroll
            for (int u = 0; u < U; u++) {
                double v[3], wt, er;
                value(m[u], r[u], v, wt, er);
                if (!in[u]) wt = er = 0.0;
                add(v, wt, er);
                if (pj)                                    // (tile mode: no packed slices)
#pragma unroll
                    for (int a = 0; a < 3; a++) pj[a * n + kk[u]] = (JT)v[a];
            }
            k += U * 64;
        };
        using I4 = std::integral_constant<int, 4>;
        if constexpr (GU == 4) {
            while (k + 3 * 64 < k1) step(I4{}, false);
        } else if constexpr (GU == 6) {
            while (k + 5 * 64 < k1) step(std::integral_constant<int, 6>{}, false);
            if (k + 4 * 64 < k1) step(std::integral_constant<int, 6>{}, true);   // 5 left
        } else {
            while (k + 7 * 64 < k1) step(std::integral_constant<int, 8>{}, false);
            if (k + 4 * 64 < k1) step(std::integral_constant<int, 8>{}, true);   // 5..7 left
        }
        if (k < k1) step(I4{}, true);                                             // 1..4 left
        if (G.wsplit[w]) {                             // lane pairs: lane j's sums + lane j + 32's
#pragma unroll
            for (int k = 0; k < 6; k++) H[k] += __shfl_xor(H[k], 32);
#pragma unroll
            for (int a = 0; a < 3; a++) bb[a] += __shfl_xor(bb[a], 32);
        }
        if (l >= 0) {
#pragma unroll
            for (int k = 0; k < 6; k++) { G.Hv[6 * (int64_t)l + k] = H[k]; G.Dv[6 * (int64_t)l + k] = D[k]; }
            const int64_t o = G.hd + 3 * (int64_t)(G.row0 + l);
#pragma unroll
            for (int a = 0; a < 3; a++) G.b[o + a] = bb[a];
            mx = fmax(fabs(H[0]), fmax(fabs(H[2]), fabs(H[5])));
        }
    }
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0 && lb < max(G.nrb2, 1)) G.mpart[lb] = fmax(fmax(red4[0], red4[1]), fmax(red4[2], red4[3]));
}

// heavy vertices' H / b partials per phase-1 block (owned ARAP edges: lower 6x6 + 6; depth: 1 + 1);
// one workgroup per group of blocks (G.glb: consecutive owned ARAP blocks of one pair, their edges
// contiguous) — the group's sums land in its first block's partial, its other blocks' are zero
__global__ void __launch_bounds__(256) k_sp_glin_blocks(const SpDev G) {
    __shared__ double red[kSpLin][4];
    if (gated_off(G.lgate)) return;
    const int2 gr = G.glb[blockIdx.x];
    const int4 d = G.blk[gr.x];
    const int kind = d.x & 0xff, owned = d.x >> 8;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = d.z + threadIdx.x;
    double *out = G.lpart + (int64_t)kSpLin * gr.x;
    if (kind == SP_ARAP) {
        if (!owned) return;
        double a[kSpLin];
#pragma unroll
        for (int k = 0; k < kSpLin; k++) a[k] = 0.0;
        const int iend = G.blk[gr.x + gr.y - 1].w;
        for (int ii = i; ii < iend; ii += 256) {
            double J[6];
#pragma unroll
            for (int r = 0; r < 6; r++) J[r] = G.Ja[(12 + r) * G.jld + ii];
            const double wv = G.Wa[ii], er = G.Ea[ii];
#pragma unroll
            for (int r = 0; r < 6; r++) {
                const double jr = J[r] * wv;
#pragma unroll
                for (int c = 0; c <= r; c++) a[tri6(r, c)] += jr * J[c];
                a[21 + r] -= J[r] * (wv * er);
            }
        }
        for (int k = threadIdx.x; k < kSpLin * (gr.y - 1); k += 256) out[kSpLin + k] = 0.0;
#pragma unroll
        for (int k = 0; k < kSpLin; k++) {
            const double v = wave_sum(a[k]);
            if (lane == 0) red[k][w] = v;
        }
        __syncthreads();
        if (threadIdx.x < kSpLin) {
            const int k = threadIdx.x;
            out[k] = (red[k][0] + red[k][1]) + (red[k][2] + red[k][3]);
        }
    } else {
        double h = 0.0, bs = 0.0;
        if (i < d.w) {
            const int le = G.dperm[i];
            const double js = G.Jd[4 * (int64_t)le + 3];
            h = G.wss[le];
            bs = -js * (G.Wd[le] * G.Ed[le]);
        }
        h = wave_sum(h);
        bs = wave_sum(bs);
        if (lane == 0) { red[0][w] = h; red[1][w] = bs; }
        __syncthreads();
        if (threadIdx.x < 2) {
            const int k = threadIdx.x;
            out[k] = (red[k][0] + red[k][1]) + (red[k][2] + red[k][3]);
        }
    }
}

// heavy H / b (rank sums) in two levels: one workgroup per chunk of a heavy vertex's block partials
// (kSpHeavyChunk of them; thread (g, c) = (tid / 32, tid % 32) adds value c of every 8th partial,
// the 8 groups added in order), then the vertex's last chunk to finish adds its chunks' sums in order
// (same hand-off as the CG chain's last workgroups: coherent stores, a ticket per vertex)
__global__ void __launch_bounds__(256) k_sp_glin_heavy(const SpDev G) {
    __shared__ double lds[8][32];
    __shared__ int last;
    if (gated_off(G.lgate)) return;
    const int ch = blockIdx.x, h = G.ch_h[ch];
    const int dim = h < G.Q ? kSpLin : 2;
    const int c = threadIdx.x & 31, g = threadIdx.x >> 5;
    double acc = 0.0;
    if (c < dim) {
        int64_t k = G.ch_lo[ch] + g;
        const int64_t k1 = G.ch_lo[ch + 1];
        for (; k + 7 * 8 < k1; k += 64) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = G.lpart[(int64_t)kSpLin * G.hv_blk[k + 8 * u] + c];
#pragma unroll
            for (int u = 0; u < 8; u++) acc += v[u];
        }
        for (; k < k1; k += 8) acc += G.lpart[(int64_t)kSpLin * G.hv_blk[k] + c];
    }
    lds[g][c] = acc;
    __syncthreads();
    if ((int)threadIdx.x < dim) {
        double t = 0.0;
#pragma unroll
        for (int gg = 0; gg < 8; gg++) t += lds[gg][threadIdx.x];
        publish(G.chpart + (int64_t)kSpLin * ch + threadIdx.x, t);
    }
    const int c0 = G.hch_off[h], c1 = G.hch_off[h + 1];
    if (threadIdx.x == 0) {
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_s_waitcnt(0);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        last = __hip_atomic_fetch_add(G.hcnt + h, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == c1 - c0 - 1;
    }
    __syncthreads();
    if (!last) return;
    acc = 0.0;
    if (c < dim)
        for (int j = c0 + g; j < c1; j += 8) acc += fetch(G.chpart + (int64_t)kSpLin * j + c);
    __syncthreads();
    lds[g][c] = acc;
    __syncthreads();
    if ((int)threadIdx.x < dim) {
        double t = 0.0;
#pragma unroll
        for (int gg = 0; gg < 8; gg++) t += lds[gg][threadIdx.x];
        const int q = threadIdx.x;
        if (h < G.Q) {
            if (q < 21) G.hl[21 * (int64_t)h + q] = t;
            else G.b[6 * (int64_t)h + q - 21] = t;
        } else {
            if (q == 0) G.hl[21 * (int64_t)G.Q + (h - G.Q)] = t;
            else G.b[6 * (int64_t)G.Q + (h - G.Q)] = t;
        }
    }
    if (threadIdx.x == 0) st_sc1(G.hcnt + h, 0);
}

// rank max of the rows' diagonal (stage 0), or that (all-reduced) combined with the heavy diagonal
__global__ void __launch_bounds__(256) k_sp_maxdiag(const SpDev G, double *out, int stage) {
    __shared__ double red4[4];
    if (gated_off(G.lgate)) return;
    double m = 0.0;
    if (stage == 0) {
        for (int i = threadIdx.x; i < G.nrb2; i += 256) m = fmax(m, G.mpart[i]);
    } else {
        for (int h = threadIdx.x; h < G.Q; h += 256)
#pragma unroll
            for (int a = 0; a < 6; a++) m = fmax(m, fabs(G.hl[21 * (int64_t)h + tri6(a, a)]));
        for (int s = threadIdx.x; s < G.S; s += 256) m = fmax(m, fabs(G.hl[21 * (int64_t)G.Q + s]));
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        const double v = fmax(fmax(red4[0], red4[1]), fmax(red4[2], red4[3]));
        out[0] = stage == 0 ? v : fmax(out[0], v);
    }
}

__global__ void k_sp_cvt_j(const double *__restrict__ J, float *__restrict__ J32, int64_t n, const int *gate) {
    if (gated_off(gate)) return;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) J32[i] = (float)J[i];
}

// ---- CG ---------------------------------------------------------------------------------------------
// (3x3 SPD, lower packed) -> inverse (lower packed) through its Cholesky factor; false if not SPD
__device__ __forceinline__ bool inv3(const double *A, double lam, double *M) {
    const double a00 = A[0] + lam, a10 = A[1], a11 = A[2] + lam, a20 = A[3], a21 = A[4], a22 = A[5] + lam;
    if (!(a00 > 0.0)) return false;
    const double l00 = sqrt(a00), l10 = a10 / l00, l20 = a20 / l00;
    const double d1 = a11 - l10 * l10;
    if (!(d1 > 0.0)) return false;
    const double l11 = sqrt(d1), l21 = (a21 - l20 * l10) / l11;
    const double d2 = a22 - l20 * l20 - l21 * l21;
    if (!(d2 > 0.0)) return false;
    const double l22 = sqrt(d2);
    // L^-1 (lower)
    const double i00 = 1.0 / l00, i11 = 1.0 / l11, i22 = 1.0 / l22;
    const double i10 = -l10 * i00 * i11;
    const double i21 = -l21 * i11 * i22;
    const double i20 = -(l20 * i00 + l21 * i10) * i22;
    // M = L^-T L^-1
    M[0] = i00 * i00 + i10 * i10 + i20 * i20;
    M[1] = i11 * i10 + i21 * i20;
    M[2] = i11 * i11 + i21 * i21;
    M[3] = i22 * i20;
    M[4] = i22 * i21;
    M[5] = i22 * i22;
    return true;
}

__device__ __forceinline__ void mul3(const double *M, const double r[3], double z[3]) {
    z[0] = M[0] * r[0] + M[1] * r[1] + M[3] * r[2];
    z[1] = M[1] * r[0] + M[2] * r[1] + M[4] * r[2];
    z[2] = M[3] * r[0] + M[4] * r[1] + M[5] * r[2];
}

// 6x6 SPD (lower packed, + lam on the diagonal) -> full inverse (row-major 36); false if not SPD
__device__ bool inv6(const double *Hl, double lam, double *Mo) {
    double L[36];
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) L[i * 6 + j] = j <= i ? Hl[tri6(i, j)] + (i == j ? lam : 0.0) : 0.0;
    for (int j = 0; j < 6; j++) {
        double s = L[j * 6 + j];
        for (int k = 0; k < j; k++) s -= L[j * 6 + k] * L[j * 6 + k];
        if (!(s > 0.0)) return false;
        s = sqrt(s);
        L[j * 6 + j] = s;
        for (int i = j + 1; i < 6; i++) {
            double t = L[i * 6 + j];
            for (int k = 0; k < j; k++) t -= L[i * 6 + k] * L[j * 6 + k];
            L[i * 6 + j] = t / s;
        }
    }
    for (int c = 0; c < 6; c++) {
        double y[6];
        for (int i = 0; i < 6; i++) {
            double t = i == c ? 1.0 : 0.0;
            for (int k = 0; k < i; k++) t -= L[i * 6 + k] * y[k];
            y[i] = t / L[i * 6 + i];
        }
        for (int i = 5; i >= 0; i--) {
            double t = y[i];
            for (int k = i + 1; k < 6; k++) t -= L[k * 6 + i] * y[k];
            y[i] = t / L[i * 6 + i];
        }
        for (int i = 0; i < 6; i++) Mo[i * 6 + c] = y[i];
    }
    return true;
}

// pub: 0 plain stores; 1 partials for a last-workgroup hand-off (agent-scope stores)
__device__ __forceinline__ void pair_tree(double a0, double a1, double (*red)[4], double *out, int pub = 0) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    a0 = wave_sum(a0);
    a1 = wave_sum(a1);
    if (lane == 0) { red[0][w] = a0; red[1][w] = a1; }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double s0 = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
        const double s1 = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
        if (pub == 1) {        // partials for a last-workgroup hand-off (publish)
            st_sc1(out, s0);
            st_sc1(out + 1, s1);
        } else {
            out[0] = s0;
            out[1] = s1;
        }
    }
}

// call with every thread after thread 0 published the workgroup's partials; true in the last one
__device__ __forceinline__ bool last_block(const SpDev &G, int *cnt) {
    __shared__ int last;
    if (threadIdx.x == 0) {
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_s_waitcnt(0);             // the published stores acknowledged
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        last = ticket_last(cnt, (int)gridDim.x, (int)blockIdx.x);
    }
    __syncthreads();
    return last;
}

// Merged chain: a two-level fixed-order sum of NV doubles per workgroup (slot = blockIdx.x), the
// hand-off split by XCD group.  Every thread calls it after thread 0 published its workgroup's values
// at slots[NV * blockIdx.x].  The last workgroup of group x = blockIdx % 8 adds the group's slots
// (thread t those at x + 8 (t + 256 k), in k order; the threads in the block_sum order), publishes
// the group's sums into gs[NV * x] and takes a ticket on the top counter; the last of those adds the
// group sums in group order.  True in that workgroup, with tot[0 .. NV) set in thread 0.
template <int NV>
__device__ __forceinline__ bool group_sum(const SpDev &G, int *cnt, const double *slots, double *gs, double (*red)[4], double *tot) {
    __shared__ int flag;
    const int nb = (int)gridDim.x, x = (int)blockIdx.x & 7;
    const int gsize = (nb - x + 7) >> 3, ngroups = nb < 8 ? nb : 8;
    auto settle = [&] {                  // this thread's published stores acknowledged
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_s_waitcnt(0);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
    };
    if (threadIdx.x == 0) {
        settle();
        flag = __hip_atomic_fetch_add(cnt + 1 + x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1;
    }
    __syncthreads();
    if (!flag) return false;
    double a[NV];
#pragma unroll
    for (int v = 0; v < NV; v++) a[v] = 0.0;
    for (int j = x + 8 * (int)threadIdx.x; j < nb; j += 8 * 256)
#pragma unroll
        for (int v = 0; v < NV; v++) a[v] += fetch(slots + NV * j + v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int v = 0; v < NV; v++) {
        a[v] = wave_sum(a[v]);
        if (lane == 0) red[v][w] = a[v];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int v = 0; v < NV; v++) publish(gs + NV * x + v, (red[v][0] + red[v][1]) + (red[v][2] + red[v][3]));
        st_sc1(cnt + 1 + x, 0);          // the group is done: nobody else touches its counter
        settle();
        flag = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1;
        if (flag) {
            st_sc1(cnt, 0);
#pragma unroll
            for (int v = 0; v < NV; v++) {
                double t = 0.0;
                for (int g = 0; g < ngroups; g++) t += fetch(gs + NV * g + v);
                tot[v] = t;
            }
        }
    }
    __syncthreads();
    return flag;
}

// (r.z, r.r) of iteration it from the row-block partials of the update before it (or the setup), in
// order: k_sp_dots, or the last workgroup of that update / setup on one rank
__device__ __forceinline__ void dots_block(const SpDev &G, int it, double (*red)[4]) {
    double a0 = 0.0, a1 = 0.0;
    int i = threadIdx.x;
    for (; i + 3 * 256 <= G.nrb; i += 4 * 256) {      // four pairs in flight, added in the strided order
        double v[4][2];
#pragma unroll
        for (int u = 0; u < 4; u++) { v[u][0] = fetch(G.upart + 2 * (i + 256 * u)); v[u][1] = fetch(G.upart + 2 * (i + 256 * u) + 1); }
#pragma unroll
        for (int u = 0; u < 4; u++) { a0 += v[u][0]; a1 += v[u][1]; }
    }
    for (; i <= G.nrb; i += 256) { a0 += fetch(G.upart + 2 * i); a1 += fetch(G.upart + 2 * i + 1); }
    pair_tree(a0, a1, red, G.red + (int64_t)kSpRed * it);
}

// the sd chain: own row l's dof a, (z, p) into each of its send slots
__device__ __forceinline__ void sd_send(const SpDev &G, int l, int a, double z, double p) {
    for (int k = G.snd_off[l]; k < G.snd_off[l + 1]; k++) {
        const int64_t o = 6 * (int64_t)G.snd_slot[k] + 2 * a;
        G.sbuf[o] = z;
        G.sbuf[o + 1] = p;
    }
}

// setup at lambda: row / heavy preconditioner blocks, r = rhs, z = M r, (z, p) = (z, 0), x = 0,
// partial (r.z, r.r) per row block (+ the heavy block's last, on the rank that counts the heavy dofs)
__global__ void __launch_bounds__(3 * kSpUpdRows) k_sp_setup(const SpDev G, const double *__restrict__ rhs, double lam) {
    // the row blocks as in k_sp_update: one thread per dof for the vectors, one per row for the
    // block inverse (through LDS)
    __shared__ double sM[6 * kSpUpdRows], sR[3 * kSpUpdRows];
    __shared__ double red[2][3 * kSpUpdRows / 64], dred[2][4];
    if (gated_off(G.gate)) return;
    lam = lam_of(G, lam);
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    constexpr int nw = 3 * kSpUpdRows / 64;
    double rz = 0.0, rr = 0.0;
    // workgroup 0: the heavy dofs (dispatched first: their serial work overlaps the rows); row block
    // blockIdx - 1; partial slots as in k_sp_dots (rows 0..nrb-1, heavy nrb)
    const int rb = (int)blockIdx.x - 1, slot = rb < 0 ? G.nrb : rb;
    // the CG chain's ticket counters (sites 0 and 16; this launch counts at 32) start every solve at
    // zero, whatever an earlier solve on this plan left
    if (rb < 0 && t < 32) st_sc1(G.cnt + t, 0);
    if (rb >= 0) {
        const int l0 = rb * kSpUpdRows;
        const int nrow = min(kSpUpdRows, G.nown - l0);
        const int64_t o0 = G.hd + 3 * (int64_t)(G.row0 + l0);
        const double *Hg = G.Hv + 6 * (int64_t)l0;
        if (t < 6 * nrow) sM[t] = Hg[t];
        if (t + 3 * kSpUpdRows < 6 * nrow) sM[t + 3 * kSpUpdRows] = Hg[t + 3 * kSpUpdRows];
        const double r = t < 3 * nrow ? rhs[o0 + t] : 0.0;
        sR[t] = r;
        __syncthreads();
        if (t < nrow) {
            double Hl[6], M[6];
#pragma unroll
            for (int k = 0; k < 6; k++) Hl[k] = sM[6 * t + k];
            if (!inv3(Hl, lam, M)) {
                G.rec[0] = kSpBadBlock;
#pragma unroll
                for (int k = 0; k < 6; k++) M[k] = 0.0;
            }
#pragma unroll
            for (int k = 0; k < 6; k++) sM[6 * t + k] = M[k];
        }
        __syncthreads();
        double *Mg = G.Mv + 6 * (int64_t)l0;
        if (t < 6 * nrow) Mg[t] = sM[t];
        if (t + 3 * kSpUpdRows < 6 * nrow) Mg[t + 3 * kSpUpdRows] = sM[t + 3 * kSpUpdRows];
        if (t < 3 * nrow) {
            const int row = t / 3, a = t - 3 * row;
            const double *M = sM + 6 * row;
            const int i0 = a == 0 ? 0 : a == 1 ? 1 : 3, i1 = a == 0 ? 1 : a == 1 ? 2 : 4, i2 = a == 0 ? 3 : a == 1 ? 4 : 5;
            const double *rv = sR + 3 * row;
            const double z = M[i0] * rv[0] + M[i1] * rv[1] + M[i2] * rv[2];
            G.r[o0 + t] = r;
            G.zp[o0 + t] = make_double2(z, 0.0);
            G.x[o0 + t] = 0.0;
            if (G.sd) sd_send(G, l0 + row, a, z, 0.0);
            rz = r * z;
            rr = r * r;
        }
    } else if (t < 256) {
        for (int h = t; h < G.Q + G.S; h += 256) {
            const int o = heavy_dof(G, h);
            if (h < G.Q) {
                double *M = G.Mh + 36 * (int64_t)h;
                if (!inv6(G.hl + 21 * (int64_t)h, lam, M)) {
                    G.rec[0] = kSpBadBlock;
                    for (int k = 0; k < 36; k++) M[k] = 0.0;
                }
                double r[6];
                for (int a = 0; a < 6; a++) r[a] = rhs[o + a];
                for (int a = 0; a < 6; a++) {
                    double z = 0.0;
                    for (int c = 0; c < 6; c++) z += M[a * 6 + c] * r[c];
                    G.r[o + a] = r[a];
                    G.zp[o + a] = make_double2(z, 0.0);
                    G.x[o + a] = 0.0;
                    rz += r[a] * z;
                    rr += r[a] * r[a];
                }
            } else {
                const double a = G.hl[21 * (int64_t)G.Q + (h - G.Q)] + lam;
                double m = 0.0;
                if (!(a > 0.0)) G.rec[0] = kSpBadBlock;
                else m = 1.0 / a;
                G.Mh[36 * (int64_t)G.Q + (h - G.Q)] = m;
                const double r = rhs[o], z = m * r;
                G.r[o] = r;
                G.zp[o] = make_double2(z, 0.0);
                G.x[o] = 0.0;
                rz += r * z;
                rr += r * r;
            }
        }
        if (!G.include_heavy) rz = rr = 0.0;
    }
    rz = wave_sum(rz);
    rr = wave_sum(rr);
    if (lane == 0) { red[0][wv] = rz; red[1][wv] = rr; }
    __syncthreads();
    if (t == 0) {
        double s0 = 0.0, s1 = 0.0;
#pragma unroll
        for (int k = 0; k < nw; k++) { s0 += red[0][k]; s1 += red[1][k]; }
        double *out = G.upart + 2 * slot;
        if (G.fuse) {
            st_sc1(out, s0);
            st_sc1(out + 1, s1);
        } else {
            out[0] = s0;
            out[1] = s1;
        }
    }
    // tile mode (G.tparts, the update unfused): the first product's workgroups sum the partials
    if (G.fuse && !G.tparts && last_block(G, G.cnt + 32)) {
        // (a bad block recorded by any workgroup stops every later launch through rec[0], which the
        // next launch sees; the sums formed here are then never read)
        __syncthreads();
        if (t < 256) dots_block(G, 0, dred);
    }
}

// (r.z, r.r) of iteration it from the previous update's (or the setup's) partials, in order
__global__ void __launch_bounds__(256) k_sp_dots(int it, const SpDev G) {
    __shared__ double red[2][4];
    if (gated_off(G.gate) || G.rec[0] != 0.0) return;
    dots_block(G, it, red);
}

// the sum of heavy vertex h's phase-1 block partials, component threadIdx.x (< its dim): thread
// (g, c) = (tid / 8, tid % 8) adds component c of every 32nd block partial (8 lanes read one 64-byte
// partial), then the 32 groups are added in order through LDS
__device__ __forceinline__ double heavy_part_sum(const SpDev &G, int h, double *lds) {
    const int64_t k0 = G.hv_blk_off[h], k1 = G.hv_blk_off[h + 1];
    const int dim = h < G.Q ? 6 : 1;
    const int c = threadIdx.x & 7, g = threadIdx.x >> 3;
    double acc = 0.0;
    if (c < dim) {
        int64_t k = k0 + g;
        for (; k + 7 * 32 < k1; k += 8 * 32) {        // eight partials in flight, added in order
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = G.part[(int64_t)kSpPart * G.hv_blk[k + 32 * u] + c];
#pragma unroll
            for (int u = 0; u < 8; u++) acc += v[u];
        }
        for (; k < k1; k += 32) acc += G.part[(int64_t)kSpPart * G.hv_blk[k] + c];
    }
    lds[threadIdx.x] = acc;
    __syncthreads();
    double t = 0.0;
    if ((int)threadIdx.x < dim)
        for (int gg = 0; gg < 32; gg++) t += lds[8 * gg + threadIdx.x];
    return t;
}

// heavy sums of one heavy vertex h into hbuf[1 + its dofs] (h == Q + S: p.q of the rank's rows into
// hbuf[0]), one workgroup: thread (g, c) = (tid / 8, tid % 8) adds component c of every 32nd block
// partial (8 lanes read one 64-byte partial), then the 32 groups are added in order through LDS
__device__ __forceinline__ void heavy_sums_block(const SpDev &G, int h, double *red4, double *lds) {
    const int nh = G.Q + G.S;
    if (h == nh) {
        double a = 0.0;
        int i = threadIdx.x;
        for (; i + 3 * 256 < G.nrb2; i += 4 * 256) {
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = fetch(G.rpart + i + 256 * u);
#pragma unroll
            for (int u = 0; u < 4; u++) a += v[u];
        }
        for (; i < G.nrb2; i += 256) a += fetch(G.rpart + i);
        a = block_sum(a, red4);
        if (threadIdx.x == 0) publish(G.hbuf, a);
        return;
    }
    const int o = heavy_dof(G, h);
    const double t = heavy_part_sum(G, h, lds);
    if ((int)threadIdx.x < (h < G.Q ? 6 : 1)) publish(G.hbuf + 1 + o + threadIdx.x, t);
    __syncthreads();
}

// heavy q (= sums + lam p), p formed and stored, p.q and alpha of iteration it from hbuf
__device__ __forceinline__ void heavy_finish(const SpDev &G, int it, double lam, double beta, double *red4) {
    double pqh = 0.0;
    for (int64_t dd = threadIdx.x; dd < G.hd; dd += 256) {
        const double2 v = G.zp[dd];
        const double p = __fma_rn(beta, v.y, v.x);
        const double qh = fetch(G.hbuf + 1 + dd) + lam * p;
        G.q[dd] = qh;
        G.zp[dd] = make_double2(v.x, p);
        pqh += p * qh;
    }
    pqh = block_sum(pqh, red4);
    if (threadIdx.x == 0) {
        const double pq = fetch(G.hbuf) + pqh;
        const double alpha = G.red[(int64_t)kSpRed * it] / pq;
        if (!(pq > 0.0) || !isfinite(alpha)) { G.rec[0] = kSpBreakdown; G.rec[1] = it; }
        G.red[(int64_t)kSpRed * it + 3] = alpha;
    }
}

// merged chain, phase 2: alpha of iteration it.  Workgroup 0 (dispatched first, waits on nothing)
// sums phase 1's p.Ap partials in a fixed order, records alpha (NaN on breakdown, with the stop word
// of iteration it + 1) and publishes it: the value with an agent-scope store, acknowledged, then the
// flag = it.  The other workgroups call m2_alpha_wait where they first need alpha (after their
// sums): thread 0 polls the flag, the value goes through LDS.
// The wait rests on workgroup 0 being resident while the others poll: the dispatcher hands out a
// launch's workgroups in index order, so workgroup 0 starts before any waiter; HIP does not promise
// this.  The poll is bounded: a timeout skips the workgroup's update and leaves kSpTimeout for the
// next iteration, which the host raises as an error (never a rejected trial) and answers by
// switching the context to the separate alpha launch (k_sp_alpha).  Either way every workgroup still
// draws its ticket in m2_dots, so the counters return to zero.
// the first sixteen of thread t's partials (t, t + 256, ...; zeros past the end) and r.z: phase 2's
// workgroup 0 issues these loads before its state test, so they overlap it
struct AlphaPre {
    double v[16];
    double gam;
};
__device__ __forceinline__ void m2_alpha_loads(const SpDev &G, int it, AlphaPre &pf) {
    const int n = G.m1n, j = threadIdx.x;
#pragma unroll
    for (int u = 0; u < 16; u++) pf.v[u] = j + 256 * u < n ? G.m1part[j + 256 * u] : 0.0;
    pf.gam = G.red[(int64_t)kSpRed * it];
}
// writer = false (tile mode, G.tparts: every workgroup forms alpha itself, the same sum in the same
// order): the value only, workgroup 0 records it
__device__ __forceinline__ double m2_alpha_make(const SpDev &G, int it, double *red4, bool publish, const AlphaPre &pf,
                                                bool writer = true) {
    __shared__ double sa;
    // thread t adds partials t, t + 256, ... in order; sixteen loads in flight (a C2-size launch,
    // ~3,200 partials, in one round trip: alpha is on every row's path), the missing ones as zeros
    double a = 0.0;
    const int n = G.m1n;
    const double gam = pf.gam;
#pragma unroll
    for (int u = 0; u < 16; u++) a += pf.v[u];
    for (int j = threadIdx.x + 16 * 256; j < n; j += 16 * 256) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = j + 256 * u < n ? G.m1part[j + 256 * u] : 0.0;
#pragma unroll
        for (int u = 0; u < 16; u++) a += v[u];
    }
    a = block_sum(a, red4);
    if (threadIdx.x == 0) {
        double alpha = gam / a;
        if (!(a > 0.0) || !isfinite(alpha) || alpha == 0.0) {
            if (writer) st_sc1(G.red + (int64_t)kSpRed * (it + 1) + 2, (double)kSpBreakdown);   // read from the next launch on (and m2_dots)
            alpha = __builtin_nan("");
        }
        // the value is its own flag: word 3 of iteration it's record is zero until this store (the
        // record is cleared per solve; alpha == 0 counts as a breakdown above), so a waiter polls
        // the one word — one round trip after the store instead of a flag and then the value
        if (!writer) {
        } else if (publish) {
            st_sc1(G.red + (int64_t)kSpRed * it + 3, alpha);
        } else {
            G.red[(int64_t)kSpRed * it + 3] = alpha;
        }
        sa = alpha;
    }
    __syncthreads();
    return sa;
}
__device__ __forceinline__ double m2_alpha_wait(const SpDev &G, int it) {
    __shared__ double sa;
    if (threadIdx.x == 0) {
        const double *w = G.red + (int64_t)kSpRed * it + 3;
        // a waiter polls ~2^16 times (s_sleep 2 between polls: well above the ~3 us a publish takes,
        // well below a second of stall); DEFTRI_SP_INJECT_TIMEOUT_IT forces the timeout (tests)
        int n = it == G.inj_timeout_it ? (1 << 16) : 0;
        double v = ld_sc1(w);
        while (__double_as_longlong(v) == 0 && n < (1 << 16)) {
            __builtin_amdgcn_s_sleep(2);
            v = ld_sc1(w);
            n++;
        }
        if (n >= (1 << 16)) {                          // never expected: stop the solve, skip the update
            st_sc1(G.red + (int64_t)kSpRed * (it + 1) + 2, (double)kSpTimeout);
            sa = __builtin_nan("");
        } else {
            sa = v;
        }
    }
    __syncthreads();
    return sa;
}

// merged chain, G.alpha_kernel: alpha of iteration it in a one-workgroup launch between the phases
__global__ void __launch_bounds__(256) k_sp_alpha(int it, const SpDev G) {
    __shared__ double red4[4];
    if (gated_off(G.gate)) return;
    double beta;
    if (it_state(G, it, beta)) return;
    AlphaPre pf;
    m2_alpha_loads(G, it, pf);
    m2_alpha_make(G, it, red4, false, pf);
}

// MG 1 (merged chain, one rank): also p.Ap = sum_e s_e (J_e p) + sum_dep p_s (2 c_e . p_v + W J_s^2 p_s)
// + sum_v p_v . (D_v + lam) p_v + lam |p_h|^2 per workgroup — the first m_nx workgroups do the heavy
// dofs (p_h stored for phase 2) and the row terms, 256 rows each — and alpha in the last workgroup.
// MG 2 (sharded single-reduction chain): the same sums with z in place of p (beta = 0: the product
// is A z, the partials are z.Az over the rank's owned edges, own rows and — on the rank that counts
// them — the heavy dofs); the rows' z are read through apts_p (halo rows in the receive region)
template <class JT, int MG>
__global__ void __launch_bounds__(256) k_sp_phase1(int it, const SpDev G, const JT *__restrict__ Jarap, double lam) {
    __shared__ double red[7][4];
    if (gated_off(G.gate)) return;
    lam = lam_of(G, lam);
    double beta = 0.0;
    if constexpr (MG == 2) {
        if (G.rec[0] != 0.0) return;             // the state is decided by the update (k_sp_update_sd)
    } else {
        if (it_state(G, it, beta)) return;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int bx = G.p1list ? G.p1list[blockIdx.x] : (int)blockIdx.x;    // (sharded overlap: a subset)
    if constexpr (MG) {
        double pap = 0.0;
        const int e = bx;
        if (e < G.m_nx) {
            if (e == 0) {
                for (int64_t dd = threadIdx.x; dd < G.hd; dd += 256) {
                    const double p = pval(G.zp, beta, dd);
                    G.ph[dd] = p;
                    pap += lam * (p * p);
                }
                if (!G.include_heavy) pap = 0.0;      // replicated dofs: counted on one rank
            } else if (e - 1 < G.nrb) {
                const int l = (e - 1) * 256 + (int)threadIdx.x;
                if (l < G.nown) {
                    const int64_t o = G.hd + 3 * (int64_t)(G.row0 + l);
                    double p[3], D[6];
#pragma unroll
                    for (int c = 0; c < 3; c++) p[c] = pval(G.zp, beta, o + c);
#pragma unroll
                    for (int k = 0; k < 6; k++) D[k] = G.Dv[6 * (int64_t)l + k];
                    const double q0 = lam * p[0] + ((D[0] * p[0] + D[1] * p[1]) + D[3] * p[2]);
                    const double q1 = lam * p[1] + ((D[1] * p[0] + D[2] * p[1]) + D[4] * p[2]);
                    const double q2 = lam * p[2] + ((D[3] * p[0] + D[4] * p[1]) + D[5] * p[2]);
                    pap = (p[0] * q0 + p[1] * q1) + p[2] * q2;
                }
            }
            pap = block_sum(pap, red[0]);
            if (threadIdx.x == 0) G.m1part[bx] = pap;
            return;
        }
    }
    const int b = MG ? bx - G.m_nx : bx;
    const int4 d = G.blk[b];
    const int kind = d.x & 0xff, owned = d.x >> 8;
    const int i = d.z + threadIdx.x;
    double *out = G.part + (int64_t)kSpPart * b;
    double pap = 0.0;
    if (kind == SP_ARAP) {
        double acc[6] = {0, 0, 0, 0, 0, 0};
        if (i < d.w) {
            const int4 rw = reinterpret_cast<const int4 *>(MG == 2 ? G.apts_p : G.apts)[i];
            double J[18];
#pragma unroll
            for (int k = 0; k < 18; k++) J[k] = (double)Jarap[k * G.jld + i];
            const int rows[4] = {rw.x, rw.y, rw.z, rw.w};
            double t = 0.0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int64_t o = G.hd + 3 * (int64_t)rows[k];
#pragma unroll
                for (int c = 0; c < 3; c++) t += J[3 * k + c] * pval(G.zp, beta, o + c);
            }
            const int64_t oT = 6 * (int64_t)d.y;
#pragma unroll
            for (int c = 0; c < 6; c++) t += J[12 + c] * pval(G.zp, beta, oT + c);
            const double s = G.Wa[i] * t;
            G.s[i] = s;
            if (MG && owned) pap = s * t;            // (one rank: every edge owned)
            if (owned)
#pragma unroll
                for (int c = 0; c < 6; c++) acc[c] = J[12 + c] * s;
        }
        if (!MG && !owned) return;
#pragma unroll
        for (int c = 0; c < 6; c++) {
            const double v = wave_sum(acc[c]);
            if (lane == 0) red[c][w] = v;
        }
        if (MG) {
            pap = wave_sum(pap);
            if (lane == 0) red[6][w] = pap;
        }
        __syncthreads();
        if (threadIdx.x < (MG ? 7 : 6)) {
            const int c = threadIdx.x;
            const double v = (red[c][0] + red[c][1]) + (red[c][2] + red[c][3]);
            if (c < 6) out[c] = v;
            else G.m1part[bx] = v;
        }
    } else {
        double t = 0.0;
        if (i < d.w) {
            const int le = G.dperm[i];
            const int64_t o = G.hd + 3 * (int64_t)G.drow[le];
            const double *c = G.cdep + 3 * (int64_t)le;
            const double cp = (c[0] * pval(G.zp, beta, o) + c[1] * pval(G.zp, beta, o + 1)) + c[2] * pval(G.zp, beta, o + 2);
            const double ps = pval(G.zp, beta, 6 * (int64_t)G.Q + d.y);
            t = cp + G.wss[le] * ps;
            if (MG) pap = ps * (cp + t);
        }
        t = wave_sum(t);
        if (lane == 0) red[0][w] = t;
        if (MG) {
            pap = wave_sum(pap);
            if (lane == 0) red[6][w] = pap;
        }
        __syncthreads();
        if (threadIdx.x == 0) out[0] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
        if (MG && threadIdx.x == 6) G.m1part[bx] = (red[6][0] + red[6][1]) + (red[6][2] + red[6][3]);
    }
}

// merged chain, phase 2: after every workgroup published its (r.z, r.r) partial, the last one forms
// those of iteration it + 1
__device__ __forceinline__ void m2_dots(const SpDev &G, int it, double (*red)[4]) {
    double tot[2];
    if (group_sum<2>(G, G.cnt, G.m2part, G.gsum + 16, red, tot) && threadIdx.x == 0) {
        G.red[(int64_t)kSpRed * (it + 1)] = tot[0];
        G.red[(int64_t)kSpRed * (it + 1) + 1] = tot[1];
        // the state of iteration it + 1 as the next launch's it_state would find it — the stop word
        // (stored agent-scope, settled before its workgroup's ticket), converged, budget — into the
        // record: this is the launch's last workgroup, so every other one has tested its state
        // already, and the chain needs no status-only tail launch
        if (G.rec[0] == 0.0) {
            const double sw = ld_sc1(G.red + (int64_t)kSpRed * (it + 1) + 2);
            int st = 0;
            if (sw != 0.0) st = (int)sw;
            else if (tot[1] <= G.tol2 * G.red[1]) st = kSpConverged;
            else if (it + 1 >= G.max_it) st = kSpBudget;
            if (st) { G.rec[0] = st; G.rec[1] = it + 1; }
        }
    }
}

// one wave per 64 rows of the wave layout: per slot (coalesced [k][64]) the entry's J slice times
// s_e (ARAP) or p of the depth edge's scale; then the row's own terms
// at most 4 waves per SIMD: the registers go to gathers in flight (a C2-size grid has ~3 waves per
// SIMD to hide their latency with)
// MG (merged chain, one rank): the update of iteration it follows in the same thread — x += alpha p,
// r -= alpha q, z = M r, (z, p) stored (q never is) — and the (r.z, r.r) of iteration it + 1 are
// formed by the last workgroup; the first m_nh workgroups do the heavy vertices (their sums, q, update)
// MG 2 (sharded single-reduction chain): the rows' w = A z stored into q; the first m_nh workgroups
// write this rank's part of the reduction record xb = [r.z, r.r, z.Az, heavy sums of A z]: one per
// heavy vertex its block partials' sums, then z.Az from phase 1's partials and (r.z, r.r) from the
// last update's (or the setup's) — all from earlier launches, so no hand-off; the host all-reduces xb
// U (G.p2u): slots per step of the slot loop — 8 (up to 4 waves per SIMD) or 4 (registers for 8
// waves per SIMD, for the row split's extra waves)
template <class JT, int MG, int U8>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(U8 == 4 ? 6 : 4, U8 == 4 ? 8 : 4)))
k_sp_phase2(int it, const SpDev G, double lam, const JT *__restrict__ pj) {
    __shared__ double red4[4];
    if (gated_off(G.gate)) return;
    lam = lam_of(G, lam);
    double beta = 0.0;
    if constexpr (MG == 2) {
        if (G.rec[0] != 0.0) return;
        if ((int)blockIdx.x < G.m_nh) {
            const int nh = G.Q + G.S;
            const int h = blockIdx.x;
            if (h < nh) {
                __shared__ double lds[256];
                const double t = heavy_part_sum(G, h, lds);
                if ((int)threadIdx.x < (h < G.Q ? 6 : 1)) G.xb[3 + heavy_dof(G, h) + threadIdx.x] = t;
            } else if (h == nh) {                     // z.Az: phase 1's workgroup partials, in order
                double a = 0.0;
                for (int j = threadIdx.x; j < G.m1n; j += 256) a += G.m1part[j];
                a = block_sum(a, red4);
                if (threadIdx.x == 0) G.xb[2] = a;
            } else if (h == nh + 1) {                 // (r.z, r.r): the update's row-block partials
                double a0 = 0.0, a1 = 0.0;
                for (int j = threadIdx.x; j <= G.nrb; j += 256) { a0 += G.upart[2 * j]; a1 += G.upart[2 * j + 1]; }
                a0 = block_sum(a0, red4);
                a1 = block_sum(a1, red4);
                if (threadIdx.x == 0) { G.xb[0] = a0; G.xb[1] = a1; }
            }
            return;
        }
    }
    AlphaPre pf;                                            // MG 1, workgroup 0: alpha's loads first
    if (MG == 1 && !G.alpha_kernel && blockIdx.x == 0) m2_alpha_loads(G, it, pf);
    if (MG == 2) {
    } else if (const int st = it_state(G, it, beta)) {
        // with the heavy finish folded in here, k_sp_heavy's record of the first stopped iteration too
        if ((MG || G.fuse_heavy) && blockIdx.x == 0 && threadIdx.x == 0) record_stop(G, it, st);
        return;
    }
    double alpha = 0.0;
    double pq = 0.0, rr2 = 0.0;                             // (MG: r.z and r.r)
    bool rows = true;
    int hv = -1;                                            // MG: the heavy vertex of this workgroup
    double th = 0.0;                                        // ... its component sum (thread < dim)
    if constexpr (MG == 1) {
        if (G.alpha_kernel) alpha = G.red[(int64_t)kSpRed * it + 3];     // k_sp_alpha's
        else if (blockIdx.x == 0) alpha = m2_alpha_make(G, it, red4, true, pf);
        if ((int)blockIdx.x < G.m_nh) {
            rows = false;
            if ((int)blockIdx.x < G.Q + G.S) {
                __shared__ double lds[256];
                hv = blockIdx.x;
                th = heavy_part_sum(G, hv, lds);
            }
        }
    }
    const int nhx = MG ? G.m_nh : G.fuse_heavy ? G.Q + G.S : 0;
    (void)alpha;
    if (!MG && (int)blockIdx.x < nhx) {
        // the heavy vertices' sums (phase-1 partials only): dispatched first, concurrent with the rows
        __shared__ double lds[256];
        heavy_sums_block(G, blockIdx.x, red4, lds);
        if (last_block(G, G.cnt)) {
            heavy_sums_block(G, G.Q + G.S, red4, lds);
            __syncthreads();
            heavy_finish(G, it, lam, beta, red4);
        }
        return;
    }
    // row split (G.rs = 1, 2 or 4): a workgroup's 4 waves are 4 / rs row-waves x rs parts; part j of a
    // row-wave walks the j-th contiguous share of its slot steps, and part 0 adds the others' sums
    // (through LDS, in part order) before the row's own terms — rs x the waves in flight for the
    // slot gathers, whose latency bounds this loop at ~3 waves per SIMD (C2)
    const int rpw = 4 >> (G.rs >> 1), wv = threadIdx.x >> 6;
    const int lb = rows ? row_block(blockIdx.x - nhx, G.nrb2) : 0;
    const int rw = wv & (rpw - 1), part = wv / rpw;
    const int w = lb * rpw + rw, lane = threadIdx.x & 63;
    __shared__ double qx[3][3][128];                        // parts 1..3: [part - 1][component][row lane]
    // MG: the row's values for the update after alpha arrives (lrow >= 0: this lane has a row)
    int lrow = -1;
    int64_t orow = 0;
    double pr[3] = {0, 0, 0}, qr[3] = {0, 0, 0}, xo[3] = {0, 0, 0}, ro[3] = {0, 0, 0}, M[6] = {0, 0, 0, 0, 0, 0};
    double q[3] = {0.0, 0.0, 0.0};
    int l = -1;
    if (rows && w < G.nwaves) {
        l = G.rowmap[64 * w + lane];
        const int64_t n = G.nslots * 64;
        const JT *pjx = pj, *pjy = pj + n, *pjz = pj + 2 * n;
        const int64_t os = 6 * (int64_t)G.Q;
        int64_t s0 = G.woff[w], s1 = G.woff[w + 1];
        if (G.rs > 1) {
            const int64_t per = (s1 - s0 + G.rs - 1) / G.rs;
            s0 = min(s0 + part * per, s1);
            s1 = min(s0 + per, s1);
        }
        int64_t k = s0 * 64 + lane;
        const int64_t k1 = s1 * 64 + lane;
        // s_e (v >= 0), p of the depth scale -2 - v (v <= -2) or 0 (padding): both loads on every
        // path and a select, so the slots of a step keep their loads in flight (the scales' (z, p)
        // are a handful of cache lines)
        const double *__restrict__ sv_ = G.s;
        const double2 *__restrict__ zp_ = G.zp;
        const double *__restrict__ ph_ = G.ph;
        auto val = [&](int v) -> double {
            const double a = sv_[max(v, 0)];
            if constexpr (MG) {
                // p from phase 1's copy (the heavy workgroups rewrite zp); blended arithmetically (both
                // terms finite, one factor 1 and one 0: exact) — with a select the compiler sinks this
                // load into a per-slot branch that waits on every load in flight
                const double p = ph_[os + max(-2 - v, 0)];
                return a * (v >= 0 ? 1.0 : 0.0) + p * (v <= -2 ? 1.0 : 0.0);
            } else {
                const double2 z = zp_[os + max(-2 - v, 0)];
                const double p = __fma_rn(beta, z.y, z.x);
                return v >= 0 ? a : (v <= -2 ? p : 0.0);
            }
        };
        // U slots per step: their indices, then the values and J slices, then the adds in order.  A
        // clamped step (the last, with fewer than U slots left: the count is uniform in the wave)
        // reads the last slot again in place of the missing ones and adds them times zero
        auto step = [&](auto U_, bool clamp) {
            constexpr int U = decltype(U_)::value;
            int v[U];
            int64_t kk[U];
            double sv[U], J[U][3], mk[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const bool in = k + 64 * u < k1;
                kk[u] = clamp && !in ? k1 - 64 : k + 64 * u;
                mk[u] = clamp && !in ? 0.0 : 1.0;
            }
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = G.pidx[kk[u]];
            if constexpr (MG) {
                // every load of the step first (s_e, the scale's p, the J slice), the arithmetic after:
                // one round trip per step instead of one per slot
                double a[U], pp[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    J[u][0] = pjx[kk[u]]; J[u][1] = pjy[kk[u]]; J[u][2] = pjz[kk[u]];
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    a[u] = sv_[max(v[u], 0)];
                    pp[u] = ph_[os + max(-2 - v[u], 0)];
                }
#pragma unroll
                for (int u = 0; u < U; u++)
                    sv[u] = (a[u] * (v[u] >= 0 ? 1.0 : 0.0) + pp[u] * (v[u] <= -2 ? 1.0 : 0.0)) * mk[u];
            } else {
#pragma unroll
                for (int u = 0; u < U; u++) {
                    sv[u] = val(v[u]) * mk[u];
                    J[u][0] = pjx[kk[u]]; J[u][1] = pjy[kk[u]]; J[u][2] = pjz[kk[u]];
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int a = 0; a < 3; a++) q[a] += J[u][a] * sv[u];
            k += U * 64;
        };
        if constexpr (U8 == 8) {
            while (k + 7 * 64 < k1) step(std::integral_constant<int, 8>{}, false);
            if (k + 4 * 64 < k1) step(std::integral_constant<int, 8>{}, true);   // 5..7 slots left
            else if (k < k1) step(std::integral_constant<int, 4>{}, true);      // 1..4
        } else {
            while (k + 3 * 64 < k1) step(std::integral_constant<int, 4>{}, false);
            if (k < k1) step(std::integral_constant<int, 4>{}, true);           // 1..3
        }
    }
    if (rows && w < G.nwaves && G.wsplit[w]) {          // lane pairs (wave-uniform): j's sums + j + 32's
#pragma unroll
        for (int c = 0; c < 3; c++) q[c] += __shfl_xor(q[c], 32);
    }
    if (G.rs > 1) {
        // parts 1.. hand their sums to part 0 (uniform: every workgroup of the launch passes here)
        if (part > 0) {
#pragma unroll
            for (int c = 0; c < 3; c++) qx[part - 1][c][64 * rw + lane] = q[c];
        }
        __syncthreads();
        if (part == 0)
            for (int j = 1; j < G.rs; j++)
#pragma unroll
                for (int c = 0; c < 3; c++) q[c] += qx[j - 1][c][64 * rw + lane];
    }
    if (part == 0 && l >= 0) {
        {
            const int64_t o = G.hd + 3 * (int64_t)(G.row0 + l);
            double2 v[3];
            double p[3], D[6];
#pragma unroll
            for (int c = 0; c < 3; c++) v[c] = G.zp[o + c];
#pragma unroll
            for (int k = 0; k < 6; k++) D[k] = G.Dv[6 * (int64_t)l + k];
            if constexpr (MG == 1) {
#pragma unroll
                for (int c = 0; c < 3; c++) { xo[c] = G.x[o + c]; ro[c] = G.r[o + c]; }
#pragma unroll
                for (int k = 0; k < 6; k++) M[k] = G.Mv[6 * (int64_t)l + k];
            }
#pragma unroll
            for (int c = 0; c < 3; c++) p[c] = MG == 2 ? v[c].x : __fma_rn(beta, v[c].y, v[c].x);
            q[0] += lam * p[0] + ((D[0] * p[0] + D[1] * p[1]) + D[3] * p[2]);
            q[1] += lam * p[1] + ((D[1] * p[0] + D[2] * p[1]) + D[4] * p[2]);
            q[2] += lam * p[2] + ((D[3] * p[0] + D[4] * p[1]) + D[5] * p[2]);
            if constexpr (MG == 2) {
#pragma unroll
                for (int c = 0; c < 3; c++) G.q[o + c] = q[c];          // w = A z of the row
            } else if constexpr (MG == 1) {
                lrow = l;
                orow = o;
#pragma unroll
                for (int c = 0; c < 3; c++) { pr[c] = p[c]; qr[c] = q[c]; }
            } else {
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    G.zp[o + c] = make_double2(v[c].x, p[c]);
                    G.q[o + c] = q[c];
                    pq += p[c] * q[c];
                }
            }
        }
    }
    if constexpr (MG == 2) {
        return;
    } else if constexpr (MG == 1) {
        if (!G.alpha_kernel && blockIdx.x != 0) alpha = m2_alpha_wait(G, it);
        if (hv >= 0) {
            // thread a < dim: component a of the vertex (k_sp_update's heavy arithmetic; r through
            // LDS, so no private arrays); its (r.z, r.r) terms added in component order
            __shared__ double rs[6], tz[2][6];
            const int h = hv, dim = h < G.Q ? 6 : 1, o = heavy_dof(G, h);
            const int a = isnan(alpha) ? dim : (int)threadIdx.x;     // breakdown: no update
            double p = 0.0, r = 0.0;
            if (a < dim) {
                p = G.ph[o + a];
                const double q = th + lam * p;
                G.x[o + a] += alpha * p;
                r = G.r[o + a] - alpha * q;
                G.r[o + a] = r;
                rs[a] = r;
            }
            __syncthreads();
            if (a < dim) {
                const double *Mh = h < G.Q ? G.Mh + 36 * (int64_t)h + a * 6 : G.Mh + 36 * (int64_t)G.Q + (h - G.Q);
                double z = 0.0;
                for (int c = 0; c < dim; c++) z += Mh[c] * rs[c];
                G.zp[o + a] = make_double2(z, p);
                tz[0][a] = r * z;
                tz[1][a] = r * r;
            }
            __syncthreads();
            if (threadIdx.x == 0 && !isnan(alpha))
                for (int c = 0; c < dim; c++) { pq += tz[0][c]; rr2 += tz[1][c]; }
        } else if (rows) {
            if (lrow >= 0 && !isnan(alpha)) {
                // k_sp_update's arithmetic for the row
                const int64_t o = orow;
                double r[3], z[3];
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    G.x[o + c] = xo[c] + alpha * pr[c];
                    r[c] = ro[c] - alpha * qr[c];
                }
                z[0] = M[0] * r[0] + M[1] * r[1] + M[3] * r[2];
                z[1] = M[1] * r[0] + M[2] * r[1] + M[4] * r[2];
                z[2] = M[3] * r[0] + M[4] * r[1] + M[5] * r[2];
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    G.r[o + c] = r[c];
                    G.zp[o + c] = make_double2(z[c], pr[c]);
                    pq += r[c] * z[c];              // (r.z, r.r) of iteration it + 1
                    rr2 += r[c] * r[c];
                }
            }
        }
        __shared__ double red[2][4];
        pair_tree(pq, rr2, red, G.m2part + 2 * blockIdx.x, 1);   // (kernel args never by address)
        m2_dots(G, it, red);
        return;
    }
    const double sm = block_sum(pq, red4);
    if (threadIdx.x == 0 && lb < max(G.nrb2, 1)) {
        if (G.fuse_heavy) publish(G.rpart + lb, sm);
        else G.rpart[lb] = sm;
    }
    if (G.fuse_heavy && last_block(G, G.cnt)) {
        // k_sp_heavy's finish of this iteration in the last workgroup (rows' p.q, heavy q, alpha)
        __shared__ double lds[256];
        heavy_sums_block(G, G.Q + G.S, red4, lds);
        __syncthreads();
        heavy_finish(G, it, lam, beta, red4);
    }
}

// heavy q, p.q and alpha of iteration it.  stage 0: one workgroup does all (small problems, one
// rank); 1: the rank's sums into hbuf [p.q of its rows, per heavy dof the sum of its blocks'
// partials] — one workgroup per heavy vertex (+ one for p.q) when launched with Q + S + 1 workgroups,
// else one workgroup looping over the vertices; 2: finish from hbuf (after the host's all-reduce, or
// stage 1 on one rank); 3: only the state of iteration it into the record (the tail of a chunk).
// On one rank with few heavy partials (G.fuse_heavy) the last workgroup of k_sp_phase2 does stages
// 1 and 2 instead.  Every path forms the same sums (heavy_sums_block, heavy_finish).
__global__ void __launch_bounds__(256) k_sp_heavy(int it, const SpDev G, double lam, int stage) {
    __shared__ double red4[4];
    if (gated_off(G.gate)) return;
    lam = lam_of(G, lam);
    double beta;
    const int st = it_state(G, it, beta);
    if (st || stage == 3) {
        if (st && stage != 2 && blockIdx.x == 0 && threadIdx.x == 0) record_stop(G, it, st);
        return;
    }
    __shared__ double lds[256];
    if (stage == 1 && gridDim.x > 1) {
        heavy_sums_block(G, blockIdx.x, red4, lds);
        return;
    }
    if (stage != 2) {
        for (int h = 0; h <= G.Q + G.S; h++) heavy_sums_block(G, h, red4, lds);
        if (stage == 1) return;
        __syncthreads();
    }
    heavy_finish(G, it, lam, beta, red4);
}

// x += alpha p, r -= alpha q, z = M r and the partial (r.z, r.r) of the rank's rows: one thread per
// dof, kSpUpdRows rows (3 kSpUpdRows threads) per workgroup so every vector access is coalesced; the
// rows' preconditioner blocks and the new r pass through LDS.  The workgroup after the row blocks
// does the heavy dofs.  One rank: the last workgroup forms k_sp_dots of iteration it + 1.
__global__ void __launch_bounds__(3 * kSpUpdRows) k_sp_update(int it, const SpDev G) {
    static_assert(kSpUpdRows == kSpBlock, "update workgroups are the row blocks of the (r.z, r.r) partials");
    __shared__ double sM[6 * kSpUpdRows], sR[3 * kSpUpdRows];
    __shared__ double red[2][3 * kSpUpdRows / 64], dred[2][4];
    if (gated_off(G.gate) || G.rec[0] != 0.0) return;
    const double alpha = G.red[(int64_t)kSpRed * it + 3];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    constexpr int nw = 3 * kSpUpdRows / 64;
    double rz = 0.0, rr = 0.0;
    // workgroup 0: the heavy dofs (dispatched first: their serial work overlaps the rows); row block
    // blockIdx - 1; partial slots as in k_sp_dots (rows 0..nrb-1, heavy nrb)
    const int rb = (int)blockIdx.x - 1, slot = rb < 0 ? G.nrb : rb;
    if (rb >= 0) {
        const int l0 = rb * kSpUpdRows;
        const int nrow = min(kSpUpdRows, G.nown - l0);
        const int64_t o0 = G.hd + 3 * (int64_t)(G.row0 + l0);
        const bool on = t < 3 * nrow;
        double p = 0.0, x = 0.0, r = 0.0, q = 0.0;
        if (on) {
            p = G.zp[o0 + t].y;
            x = G.x[o0 + t];
            r = G.r[o0 + t];
            q = G.q[o0 + t];
        }
        const double *Mg = G.Mv + 6 * (int64_t)l0;
        if (t < 6 * nrow) sM[t] = Mg[t];
        if (t + 3 * kSpUpdRows < 6 * nrow) sM[t + 3 * kSpUpdRows] = Mg[t + 3 * kSpUpdRows];
        x += alpha * p;
        r = r - alpha * q;
        sR[t] = r;
        __syncthreads();
        if (on) {
            const int row = t / 3, a = t - 3 * row;
            const double *M = sM + 6 * row, *rv = sR + 3 * row;
            // mul3's row a of the packed symmetric block (00 10 11 20 21 22)
            const int i0 = a == 0 ? 0 : a == 1 ? 1 : 3, i1 = a == 0 ? 1 : a == 1 ? 2 : 4, i2 = a == 0 ? 3 : a == 1 ? 4 : 5;
            const double z = M[i0] * rv[0] + M[i1] * rv[1] + M[i2] * rv[2];
            G.x[o0 + t] = x;
            G.r[o0 + t] = r;
            G.zp[o0 + t] = make_double2(z, p);
            rz = r * z;
            rr = r * r;
        }
    } else if (t < 256) {
        for (int h = t; h < G.Q + G.S; h += 256) {
            const int o = heavy_dof(G, h);
            const int dim = h < G.Q ? 6 : 1;
            double r[6], p[6];
            for (int a = 0; a < dim; a++) {
                p[a] = G.zp[o + a].y;
                G.x[o + a] += alpha * p[a];
                r[a] = G.r[o + a] - alpha * G.q[o + a];
                G.r[o + a] = r[a];
            }
            const double *M = h < G.Q ? G.Mh + 36 * (int64_t)h : G.Mh + 36 * (int64_t)G.Q + (h - G.Q);
            for (int a = 0; a < dim; a++) {
                double z = 0.0;
                for (int c = 0; c < dim; c++) z += M[a * dim + c] * r[c];
                G.zp[o + a] = make_double2(z, p[a]);
                rz += r[a] * z;
                rr += r[a] * r[a];
            }
        }
        if (!G.include_heavy) rz = rr = 0.0;
    }
    // fixed-order workgroup sums: wave butterflies, then the waves in order
    rz = wave_sum(rz);
    rr = wave_sum(rr);
    if (lane == 0) { red[0][wv] = rz; red[1][wv] = rr; }
    __syncthreads();
    if (t == 0) {
        double s0 = 0.0, s1 = 0.0;
#pragma unroll
        for (int k = 0; k < nw; k++) { s0 += red[0][k]; s1 += red[1][k]; }
        double *out = G.upart + 2 * slot;
        if (G.fuse) {
            st_sc1(out, s0);
            st_sc1(out + 1, s1);
        } else {
            out[0] = s0;
            out[1] = s1;
        }
    }
    if (G.fuse && last_block(G, G.cnt + 16)) {
        // k_sp_dots of iteration it + 1, in the last workgroup (its first 256 threads)
        __syncthreads();
        if (t < 256) dots_block(G, it + 1, dred);
    }
}

// Sharded single-reduction chain (Chronopoulos & Gear's CG): the update of iteration it from the
// all-reduced record xb = [gamma = r.z, r.r, delta = z.Az, heavy sums of A z]:
//   beta = gamma / gamma_prev, alpha = gamma / (delta - beta gamma / alpha_prev)   (it 0: beta 0, gamma / delta)
//   p = z + beta p, s = w + beta s (w = A z: rows from phase 2, heavy from xb + lam z),
//   x += alpha p, r -= alpha s, z = M r, partial (r.z, r.r); the boundary rows' (z, p) into the send
//   buffer (slots snd_off[l] .. snd_off[l + 1] of own row l).
// In exact arithmetic the iterates are CG's; the one reduction per iteration carries the next
// iteration's dots with this one's product.  The stop test (r.r <= tol^2 r0.r0, the budget,
// breakdown) is decided here from the reduced values, the same on every rank and in every workgroup;
// tail = 1 only records the state of iteration it.
__global__ void __launch_bounds__(3 * kSpUpdRows) k_sp_update_sd(int it, const SpDev G, double lam, int tail) {
    __shared__ double sM[6 * kSpUpdRows], sR[3 * kSpUpdRows];
    __shared__ double red[2][3 * kSpUpdRows / 64];
    if (gated_off(G.gate) || G.rec[0] != 0.0) return;
    lam = lam_of(G, lam);
    const double gamma = G.xb[0], rr = G.xb[1], delta = G.xb[2];
    const double rr0 = it == 0 ? rr : G.red[1];
    double beta = 0.0, alpha = 0.0;
    int st = 0;
    if (rr <= G.tol2 * rr0) st = kSpConverged;
    else if (it >= G.max_it) st = kSpBudget;
    else {
        double den = delta;
        if (it > 0) {
            beta = gamma / G.red[(int64_t)kSpRed * (it - 1)];
            den = delta - beta * gamma / G.red[(int64_t)kSpRed * (it - 1) + 3];
        }
        alpha = gamma / den;
        if (!(den > 0.0) || !isfinite(alpha) || !isfinite(beta)) st = kSpBreakdown;
    }
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (blockIdx.x == 0 && t == 0) {
        double *rk = G.red + (int64_t)kSpRed * it;
        rk[0] = gamma; rk[1] = rr; rk[3] = alpha; rk[4] = delta;
        if (st) record_stop(G, it, st);
    }
    if (st || tail) return;
    constexpr int nw = 3 * kSpUpdRows / 64;
    double rz = 0.0, rr1 = 0.0;
    const int rb = (int)blockIdx.x - 1, slot = rb < 0 ? G.nrb : rb;
    if (rb >= 0) {
        const int l0 = rb * kSpUpdRows;
        const int nrow = min(kSpUpdRows, G.nown - l0);
        const int64_t o0 = G.hd + 3 * (int64_t)(G.row0 + l0);
        const bool on = t < 3 * nrow;
        double z = 0.0, pp = 0.0, w = 0.0, sp = 0.0, x = 0.0, r = 0.0;
        if (on) {
            const double2 v = G.zp[o0 + t];
            z = v.x; pp = v.y;
            w = G.q[o0 + t];
            if (G.tile) {                              // the row's cross slots (other tiles' edges)
                const int l = l0 + t / 3, a = t - 3 * (t / 3);
                for (int k = G.txoff[l]; k < G.txoff[l + 1]; k++) w += G.xc[3 * (int64_t)k + a];
            }
            sp = G.sv[o0 + t];
            x = G.x[o0 + t];
            r = G.r[o0 + t];
        }
        const double *Mg = G.Mv + 6 * (int64_t)l0;
        if (t < 6 * nrow) sM[t] = Mg[t];
        if (t + 3 * kSpUpdRows < 6 * nrow) sM[t + 3 * kSpUpdRows] = Mg[t + 3 * kSpUpdRows];
        const double p = it > 0 ? z + beta * pp : z;
        const double s_ = it > 0 ? w + beta * sp : w;
        x += alpha * p;
        r -= alpha * s_;
        sR[t] = r;
        __syncthreads();
        if (on) {
            const int row = t / 3, a = t - 3 * row;
            const double *M = sM + 6 * row, *rv = sR + 3 * row;
            const int i0 = a == 0 ? 0 : a == 1 ? 1 : 3, i1 = a == 0 ? 1 : a == 1 ? 2 : 4, i2 = a == 0 ? 3 : a == 1 ? 4 : 5;
            const double zn = M[i0] * rv[0] + M[i1] * rv[1] + M[i2] * rv[2];
            G.x[o0 + t] = x;
            G.r[o0 + t] = r;
            G.sv[o0 + t] = s_;
            G.zp[o0 + t] = make_double2(zn, p);
            sd_send(G, l0 + row, a, zn, p);
            rz = r * zn;
            rr1 = r * r;
        }
    } else if (t < 256) {
        for (int h = t; h < G.Q + G.S; h += 256) {
            const int o = heavy_dof(G, h);
            const int dim = h < G.Q ? 6 : 1;
            double r[6], p[6];
            for (int a = 0; a < dim; a++) {
                const double2 v = G.zp[o + a];
                const double w = G.xb[3 + o + a] + lam * v.x;
                p[a] = it > 0 ? v.x + beta * v.y : v.x;
                const double s_ = it > 0 ? w + beta * G.sv[o + a] : w;
                G.sv[o + a] = s_;
                G.x[o + a] += alpha * p[a];
                r[a] = G.r[o + a] - alpha * s_;
                G.r[o + a] = r[a];
            }
            const double *M = h < G.Q ? G.Mh + 36 * (int64_t)h : G.Mh + 36 * (int64_t)G.Q + (h - G.Q);
            for (int a = 0; a < dim; a++) {
                double z = 0.0;
                for (int c = 0; c < dim; c++) z += M[a * dim + c] * r[c];
                G.zp[o + a] = make_double2(z, p[a]);
                rz += r[a] * z;
                rr1 += r[a] * r[a];
            }
        }
        if (!G.include_heavy) rz = rr1 = 0.0;
    }
    rz = wave_sum(rz);
    rr1 = wave_sum(rr1);
    if (lane == 0) { red[0][wv] = rz; red[1][wv] = rr1; }
    __syncthreads();
    if (t == 0) {
        double s0 = 0.0, s1 = 0.0;
#pragma unroll
        for (int k = 0; k < nw; k++) { s0 += red[0][k]; s1 += red[1][k]; }
        G.upart[2 * slot] = s0;
        G.upart[2 * slot + 1] = s1;
    }
}

// ---- tile mode (spcg_tile.cpp): one rank, one keyframe pair ----------------------------------------
// k_sp_tile, one workgroup per tile (XCD-dealt like the row blocks) + one for the heavy dofs (last):
//   P0  p = z + beta p_prev of the tile's rows and halo rows, and of the heavy dofs, into LDS
//   P1  per entry (one out-edge of a tile vertex; 64-entry chunks, one per wave and round):
//       t = J_e p, s = W t; the own rows' J^T s summed over the vertex's lanes (segmented scan, the
//       last lane stores them in LDS); the j rows' J^T s into their LDS slots, or (cut edge) into two
//       cross slots in HBM; p.Ap += s t; the pair's J_T^T s
//   P2  per tile row q = own + its LDS slots + (D_v + lambda) p + sum_dep c_e p_s, stored; the row
//       and depth terms of p.Ap, the depth scales' sums
//   one fixed-order workgroup sum of [p.Ap, J_T^T s (6), scale sums (2)] into m1part / part
// k_sp_tupd: the rows' cross slots added, alpha (workgroup 0, the merged chain's hand-off), the update
// x += alpha p, r -= alpha q, z = M r and the next (r.z, r.r) — phase 2's tail without its slot loop.
__device__ __forceinline__ double shfl_up_d(double v, int d) {
    int2 p = __builtin_bit_cast(int2, v);
    p.x = __shfl_up(p.x, (unsigned)d, 64);
    p.y = __shfl_up(p.y, (unsigned)d, 64);
    return __builtin_bit_cast(double, p);
}

// G.tparts: the state of CG iteration it from the (r.z, r.r) partials k_sp_tupd(it - 1) left, one per
// workgroup of its grid (it = 0: the setup's, one per row block + the heavy one) — every k_sp_tile
// workgroup forms the two sums itself, in one fixed order
// (thread t the partials t, t + 256, ...; then the block), so every workgroup takes the same branch
// without the update's two-level ticket chain (~6 dependent round trips at its end).  Workgroup 0
// writes them into iteration it's record words 0, 1 (k_sp_tupd's alpha, the next beta) and, when
// the solve stops here, the record.  The checks and their order are it_state's.
__device__ __forceinline__ int tile_state(const SpDev &G, int it, double &beta, double (*red)[4]) {
    beta = 0.0;
    // a stop recorded by an earlier launch (a queued iteration past convergence): no sums needed.  One
    // read per workgroup, so its waves take the same branch (workgroup 0 of this launch may write
    // the record while another workgroup's waves start)
    __shared__ double s_r0;
    const double *rk = G.red + (int64_t)kSpRed * it;
    // the record words the test reads after the sums, loaded with the stop word (one round trip)
    const double sw = rk[2], rr0 = G.red[1], gprev = it > 0 ? G.red[(int64_t)kSpRed * (it - 1)] : 1.0;
    if (threadIdx.x == 0) s_r0 = G.rec[0];
    __syncthreads();
    const double r0 = s_r0;
    if (r0 != 0.0) return (int)r0;
    const int n2 = it == 0 ? G.nrb + 1 : G.m_nh + row_grid(G.nrb);
    const double2 *parts = reinterpret_cast<const double2 *>(it == 0 ? G.upart : G.m2part);
    double a0 = 0.0, a1 = 0.0;
    int j = (int)threadIdx.x;
    for (; j + 3 * 256 < n2; j += 4 * 256) {
        double2 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = parts[j + 256 * u];
#pragma unroll
        for (int u = 0; u < 4; u++) { a0 += v[u].x; a1 += v[u].y; }
    }
    for (; j < n2; j += 256) {
        const double2 v = parts[j];
        a0 += v.x;
        a1 += v.y;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    a0 = wave_sum(a0);
    a1 = wave_sum(a1);
    if (lane == 0) { red[0][w] = a0; red[1][w] = a1; }
    __syncthreads();
    const double s0 = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    const double s1 = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    __syncthreads();
    int st = 0;
    if (sw != 0.0) st = (int)sw;
    else if (s1 <= G.tol2 * (it == 0 ? s1 : rr0)) st = kSpConverged;
    else if (it >= G.max_it) st = kSpBudget;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        G.red[(int64_t)kSpRed * it] = s0;
        G.red[(int64_t)kSpRed * it + 1] = s1;
        if (st) record_stop(G, it, st);
    }
    if (!st && it > 0) beta = s0 / gprev;
    return st;
}

// heavy vertex h's sum over the tile workgroups' partials (pair: components 0..5, scale s: 6 + s):
// thread (g, c) = (tid / 8, tid % 8) adds component c of every 32nd partial, the 32 groups in order
__device__ __forceinline__ double tile_heavy_sum(const SpDev &G, int h, double *lds, bool coherent = false) {
    const int nb = G.t_grid - 1;
    const int dim = h < G.Q ? 6 : 1;
    const int c = threadIdx.x & 7, g = threadIdx.x >> 3;
    double acc = 0.0;
    if (G.tmulti) {
        // several pairs: pair q's tiles t = tpoff[q] .. tpoff[q + 1] - 1 (workgroup b = 8 (t % seg) +
        // t / seg, the inverse of the tiles' XCD dealing); a scale s is component 6 + (s & 1) of pair s / 2
        const int q = h < G.Q ? h : (h - G.Q) >> 1, off = h < G.Q ? 0 : 6 + ((h - G.Q) & 1);
        const int seg = (G.ntile + 7) / 8, t1 = G.tpoff[q + 1];
        if (c < dim)
            for (int t = G.tpoff[q] + g; t < t1; t += 32) {
                const double *p = G.part + (int64_t)kSpPart * (8 * (t % seg) + t / seg) + off + c;
                acc += coherent ? fetch(p) : *p;
            }
    } else if (c < dim) {
        const int off = h < G.Q ? 0 : 6 + (h - G.Q);
        int k = g;
        for (; k + 7 * 32 < nb; k += 8 * 32) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const double *q = G.part + (int64_t)kSpPart * (k + 32 * u) + off + c;
                v[u] = coherent ? fetch(q) : *q;
            }
#pragma unroll
            for (int u = 0; u < 8; u++) acc += v[u];
        }
        for (; k < nb; k += 32) {
            const double *q = G.part + (int64_t)kSpPart * k + off + c;
            acc += coherent ? fetch(q) : *q;
        }
    }
    lds[threadIdx.x] = acc;
    __syncthreads();
    double t = 0.0;
    if ((int)threadIdx.x < dim)
        for (int gg = 0; gg < 32; gg++) t += lds[8 * gg + threadIdx.x];
    return t;
}

template <class JT, int SD = 0>
__global__ void __launch_bounds__(256) k_sp_tile(int it, const SpDev G, const JT *__restrict__ Jarap, double lam) {
    extern __shared__ double lds[];
    __shared__ double red[9][4];
    if (gated_off(G.gate)) return;
    lam = lam_of(G, lam);
    // everything that does not depend on the CG state is loaded before the state test's sums, so
    // those round trips overlap: the tile's table row; its rows' and halo rows' (z, p) (two per
    // thread); the heavy dofs' (z, p); the meta and chunk words of its first two entry passes; its
    // own row's slot range and depth-coupling range.  In the entry loop the meta of the pass after
    // the next is requested before the current pass is processed.
    // (sharded overlap: the launch runs a subset of the logical workgroups, G.p1list)
    const int b = G.p1list ? G.p1list[blockIdx.x] : (int)blockIdx.x, tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const bool heavy_wg = b == G.t_grid - 1;
    const int seg = (G.ntile + 7) / 8;
    const int t = heavy_wg ? G.ntile : (b & 7) * seg + (b >> 3);
    int r0 = 0, nr = 0, nh = 0, e0 = 0, ne = 0, h0 = 0, ns = 0, tq = 0;
    // own row i of the tile (local row index): consecutive from r0, or (several pairs) listed
    auto own_row = [&](int i) { return G.tmulti ? (G.trow[r0 + i] & 0x7fffffff) : G.row0 + r0 + i; };
    double2 zpre[3] = {make_double2(0.0, 0.0), make_double2(0.0, 0.0), make_double2(0.0, 0.0)};
    double2 zpre2[3] = {make_double2(0.0, 0.0), make_double2(0.0, 0.0), make_double2(0.0, 0.0)};
    double2 hz = make_double2(0.0, 0.0);
    uint2 mA = make_uint2(0u, 0u), mB = mA;     // the meta of passes 0, 1
    int2 cA = make_int2(0, 0), cB = cA;
    int rsi = 0, dj0 = 0, dj1 = 0;
    // several pairs: the own row's depth coupling in the tile's pair (G.tdep) and its diagonal block
    // loaded here too, so P2 waits on no load of its own (C3 / C5 products -2 to -3 %; one pair: the
    // same loads in P2 measured 0.5 us faster at C2)
    int dsc0 = -1;
    double cd0[3] = {0.0, 0.0, 0.0}, ws0 = 0.0, Dp[6] = {0, 0, 0, 0, 0, 0};
    if (t < G.ntile) {
        const int32_t *T = G.ttab + 8 * (int64_t)t;
        r0 = T[0]; nr = T[1]; nh = T[2]; e0 = T[3]; ne = T[4]; h0 = T[5]; ns = T[6]; tq = T[7];
        // (zp rows: own rows at row0 + local, halo rows as the upload mapped them — another rank's in
        // the receive region)
        if (tid < nr + nh) {
            const int row = tid < nr ? own_row(tid) : G.thalo[h0 + tid - nr];
            const int64_t o = G.hd + 3 * (int64_t)row;
#pragma unroll
            for (int c = 0; c < 3; c++) zpre[c] = G.zp[o + c];
        }
        if (tid + 256 < nr + nh) {
            const int i = tid + 256;
            const int row = i < nr ? own_row(i) : G.thalo[h0 + i - nr];
            const int64_t o = G.hd + 3 * (int64_t)row;
#pragma unroll
            for (int c = 0; c < 3; c++) zpre2[c] = G.zp[o + c];
        }
        // the pair's T_g (6) and its two scales: dofs 6 q .. 6 q + 5, 6 Q + 2 q, 6 Q + 2 q + 1
        const int hdof = tid < 6 ? 6 * tq + tid : 6 * G.Q + 2 * tq + tid - 6;
        if (tid < 8 && hdof < G.hd) hz = G.zp[hdof];
        const int64_t k0 = (int64_t)e0 + tid;
        if (tid < ne) { mA = G.tmeta[k0]; cA = G.tchunk[k0 >> 6]; }
        if (tid + 256 < ne) { mB = G.tmeta[k0 + 256]; cB = G.tchunk[(k0 + 256) >> 6]; }
        if (tid < nr) {
            const int l = G.tmulti ? own_row(tid) : r0 + tid;
            rsi = G.trs[r0 + tid];
            if (G.tmulti) {
                const int tdv = G.tdep[r0 + tid];
                if (tdv >= 0) {
                    const int jd = tdv >> 1;
                    dsc0 = tdv & 1;
#pragma unroll
                    for (int c = 0; c < 3; c++) cd0[c] = G.cdep[3 * (int64_t)jd + c];
                    ws0 = G.wss[jd];
                }
                if (G.trow[r0 + tid] < 0)
#pragma unroll
                    for (int kk = 0; kk < 6; kk++) Dp[kk] = G.Dv[6 * (int64_t)l + kk];
            } else {
                dj0 = G.dep_off[l];
                dj1 = G.dep_off[l + 1];
            }
        }
    }
    double beta;
    if (G.sd) {
        // sharded single-reduction chain: the product is A z (beta 0); the state is the update's
        beta = 0.0;
        if (G.rec[0] != 0.0) return;
    } else if (G.tparts) {
        if (tile_state(G, it, beta, reinterpret_cast<double(*)[4]>(&red[0][0]))) return;
    } else if (it_state(G, it, beta)) {
        return;
    }
    double pap = 0.0, jts[6] = {0, 0, 0, 0, 0, 0}, sacc[2] = {0, 0};
    if (heavy_wg) {                                // the heavy dofs: p for the update, lambda |p_h|^2
        for (int64_t dd = tid; dd < G.hd; dd += 256) {
            const double p = pval(G.zp, beta, dd);
            G.ph[dd] = p;
            pap += lam * (p * p);
        }
        if (!G.include_heavy) pap = 0.0;
        pap = block_sum(pap, red[0]);
        if (tid == 0) G.m1part[b] = pap;
        return;
    }
    if (t < G.ntile) {
        double *pL = lds, *up = pL + 3 * (nr + nh), *rs = up + 3 * nr, *hp = rs + 3 * ns;
        const int64_t jld = G.jld;
        const uint64_t lt = (1ull << lane) - 1;
        if (tid < nr + nh)
#pragma unroll
            for (int c = 0; c < 3; c++) pL[3 * tid + c] = __fma_rn(beta, zpre[c].y, zpre[c].x);   // pval
        if (tid + 256 < nr + nh)
#pragma unroll
            for (int c = 0; c < 3; c++) pL[3 * (tid + 256) + c] = __fma_rn(beta, zpre2[c].y, zpre2[c].x);
        for (int i = tid + 512; i < nr + nh; i += 256) {
            const int row = i < nr ? own_row(i) : G.thalo[h0 + i - nr];
            const int64_t o = G.hd + 3 * (int64_t)row;
#pragma unroll
            for (int c = 0; c < 3; c++) pL[3 * i + c] = pval(G.zp, beta, o + c);
        }
        for (int i = tid; i < 3 * nr; i += 256) up[i] = 0.0;
        if (tid < 8) hp[tid] = __fma_rn(beta, hz.y, hz.x);     // T_g (6), scales (<= 2); 0 past hd
        __syncthreads();
        const double W = G.pinfo[tq];              // W of every ARAP edge of the pair (k_lin_arap: W = Omega)
        for (int base = 0; base < ne; base += 256) {
            if (base + 64 * wv >= ne) break;       // (ne is a multiple of 64: whole waves in or out)
            const uint2 m = mA;
            const int2 ch = cA;
            // the next pass's meta moves up; the meta of the pass after it is requested now
            mA = mB; cA = cB;
            const int64_t k2 = (int64_t)e0 + base + 512 + tid;
            if (base + 512 + tid < ne) { mB = G.tmeta[k2]; cB = G.tchunk[k2 >> 6]; }
            else { mB = make_uint2(0u, 0u); cB = make_int2(0, 0); }
            const bool valid = (m.x & kTmValid) != 0, cut = (m.x & kTmCut) != 0;
            const bool foreign = (m.x & kTmForeign) != 0, drop = (m.x & kTmDrop) != 0;   // (sharded plans)
            const uint64_t vm = __ballot(valid), cm = __ballot(valid && cut), hm = __ballot((m.x & kTmHead) != 0);
            const int le = ch.x + __popcll(vm & lt);
            double J[18];
#pragma unroll
            for (int c = 0; c < 18; c++) J[c] = valid ? (double)Jarap[c * jld + le] : 0.0;
            const int ub = (int)(m.y >> 24), sw = (int)((m.x >> 26) & 1u);
            const int ra = valid ? ub + sw : 0, rb = valid ? ub + 1 - sw : 0;
            const int rj0 = valid ? (int)(m.x & 0xfffu) : 0, rj1 = valid ? (int)((m.x >> 12) & 0xfffu) : 0;
            // a halo-only entry: its i rows in the j fields, its j rows at ub / swap
            const int rows[4] = {foreign ? rj0 : ra, foreign ? rj1 : rb, foreign ? ra : rj0, foreign ? rb : rj1};
            double tt = 0.0;
#pragma unroll
            for (int kk = 0; kk < 4; kk++)
#pragma unroll
                for (int c = 0; c < 3; c++) tt += J[3 * kk + c] * pL[3 * rows[kk] + c];
#pragma unroll
            for (int c = 0; c < 6; c++) tt += J[12 + c] * hp[c];
            const double s = W * tt;
            if (!foreign) {                        // (an owned edge's terms count on its owner only)
                pap += s * tt;
#pragma unroll
                for (int c = 0; c < 6; c++) jts[c] += J[12 + c] * s;
            }
            if (valid && !drop) {
                if (cut) {                         // the two cross slots, at their rows' positions
                    const int2 xd = G.txdst[(int64_t)ch.y / 2 + __popcll(cm & lt)];
#pragma unroll
                    for (int c = 0; c < 3; c++) {
                        G.xc[3 * (int64_t)xd.x + c] = J[6 + c] * s;
                        G.xc[3 * (int64_t)xd.y + c] = J[9 + c] * s;
                    }
                } else {
                    const int s0 = (int)(m.y & 0xfffu), s1 = (int)((m.y >> 12) & 0xfffu);
#pragma unroll
                    for (int c = 0; c < 3; c++) { rs[3 * s0 + c] = J[6 + c] * s; rs[3 * s1 + c] = J[9 + c] * s; }
                }
            }
            // the vertex's own rows: inclusive segmented scan over its lanes (segments start at head
            // lanes; a vertex's lanes are consecutive and never cross the chunk), the last lane stores
            double v[6];
#pragma unroll
            for (int c = 0; c < 6; c++) v[c] = J[c] * s;
            const int sstart = 63 - __clzll(hm & (lt | (1ull << lane)));
            for (int d = 1; d < G.tile_segmax; d <<= 1) {
#pragma unroll
                for (int c = 0; c < 6; c++) {
                    const double y = shfl_up_d(v[c], d);
                    if (lane - d >= sstart) v[c] += y;
                }
            }
            if (valid && (m.x & kTmLast)) {
#pragma unroll
                for (int c = 0; c < 3; c++) { up[3 * ra + c] = v[c]; up[3 * rb + c] = v[3 + c]; }
            }
        }
        __syncthreads();
        if (tid < nr) {
            // several pairs: the row's home tile adds its diagonal terms and stores q, every other
            // tile of the row stores its share (its pair's sums) in the row's cross slot
            const int l = G.tmulti ? own_row(tid) : r0 + tid;
            const bool home = !G.tmulti || G.trow[r0 + tid] < 0;
            const int64_t o = G.hd + 3 * (int64_t)(G.row0 + l);
            double q[3], p[3];
#pragma unroll
            for (int c = 0; c < 3; c++) { q[c] = up[3 * tid + c]; p[c] = pL[3 * tid + c]; }
            const int sb = rsi & 0xffff, sc = rsi >> 16;
            for (int kk = sb; kk < sb + sc; kk++)
#pragma unroll
                for (int c = 0; c < 3; c++) q[c] += rs[3 * kk + c];
            if (home) {
                double D[6];
#pragma unroll
                for (int kk = 0; kk < 6; kk++) D[kk] = G.tmulti ? Dp[kk] : G.Dv[6 * (int64_t)l + kk];
                const double q0 = lam * p[0] + ((D[0] * p[0] + D[1] * p[1]) + D[3] * p[2]);
                const double q1 = lam * p[1] + ((D[1] * p[0] + D[2] * p[1]) + D[4] * p[2]);
                const double q2 = lam * p[2] + ((D[3] * p[0] + D[4] * p[1]) + D[5] * p[2]);
                pap += (p[0] * q0 + p[1] * q1) + p[2] * q2;
                q[0] += q0; q[1] += q1; q[2] += q2;
            }
            // the depth couplings: several pairs, the row's one in the tile's pair (G.tdep, loaded
            // above with its scale 2 tq or 2 tq + 1); one pair, the row's in order
            const int jend = G.tmulti ? (dsc0 >= 0 ? 1 : 0) : dj1 - dj0;
            for (int jj = 0; jj < jend; jj++) {
                const int j = dj0 + jj;
                const bool pre = G.tmulti != 0;
                const int sc_ = pre ? dsc0 : G.dsc[j];
                double cd[3];
#pragma unroll
                for (int c = 0; c < 3; c++) cd[c] = pre ? cd0[c] : G.cdep[3 * (int64_t)j + c];
                const double wsj = pre ? ws0 : G.wss[j];
                const double ps = hp[6 + sc_];
                const double cp = (cd[0] * p[0] + cd[1] * p[1]) + cd[2] * p[2];
                const double td = cp + wsj * ps;
                pap += ps * (cp + td);
                if (sc_ == 0) sacc[0] += td;
                else sacc[1] += td;
#pragma unroll
                for (int c = 0; c < 3; c++) q[c] += cd[c] * ps;
            }
            if (home) {
#pragma unroll
                for (int c = 0; c < 3; c++) G.q[o + c] = q[c];
            } else {                               // share j > 0: plane j - 1
                const int64_t x = 3 * ((int64_t)(G.tdst[r0 + tid] - 1) * G.nown + l);
#pragma unroll
                for (int c = 0; c < 3; c++) G.qs[x + c] = q[c];
            }
        }
    }
    // [p.Ap, J_T^T s, scale sums]: wave butterflies, then the waves in order
    double a[9] = {pap, jts[0], jts[1], jts[2], jts[3], jts[4], jts[5], sacc[0], sacc[1]};
#pragma unroll
    for (int kk = 0; kk < 9; kk++) {
        const double v = wave_sum(a[kk]);
        if (lane == 0) red[kk][wv] = v;
    }
    __syncthreads();
    if (tid < 9) {
        const double v = (red[tid][0] + red[tid][1]) + (red[tid][2] + red[tid][3]);
        if (tid == 0) G.m1part[b] = v;
        else G.part[(int64_t)kSpPart * b + tid - 1] = v;
    }
}

// FIN 0: the CG update of iteration it (merged-chain hand-off); FIN 1: the product only — q of every
// row (its cross slots added) and of the heavy dofs stored (the iterative plan's Hessian product)
template <int FIN>
__global__ void __launch_bounds__(256) k_sp_tupd(int it, const SpDev G, double lam, int last) {
    __shared__ double red4[4];
    if (gated_off(G.gate)) return;
    lam = lam_of(G, lam);
    double beta = 0.0;
    AlphaPre pf;
    // G.tparts: every workgroup forms alpha from the product's partials (no hand-off wait)
    const bool own_alpha = !FIN && !G.alpha_kernel && (G.tparts || blockIdx.x == 0);
    if (own_alpha) m2_alpha_loads(G, it, pf);
    if (const int st = it_state(G, it, beta)) {
        if (!FIN && blockIdx.x == 0 && threadIdx.x == 0) record_stop(G, it, st);
        return;
    }
    double alpha = 0.0, pq = 0.0, rr2 = 0.0;
    if (!FIN) {
        if (G.alpha_kernel) alpha = G.red[(int64_t)kSpRed * it + 3];
        else if (own_alpha) alpha = m2_alpha_make(G, it, red4, !G.tparts, pf, blockIdx.x == 0);
    }
    if ((int)blockIdx.x < G.m_nh) {
        __shared__ double lds[256];
        __shared__ double rsh[6], tz[2][6];
        const int h = blockIdx.x;
        const bool has = h < G.Q + G.S;
        const double th = has ? tile_heavy_sum(G, h, lds) : 0.0;
        if (!FIN && !own_alpha && !G.alpha_kernel) alpha = m2_alpha_wait(G, it);
        if (has) {
            const int dim = h < G.Q ? 6 : 1, o = heavy_dof(G, h);
            const int a = (!FIN && isnan(alpha)) ? dim : (int)threadIdx.x;
            double p = 0.0, r = 0.0;
            if (a < dim) {
                p = G.ph[o + a];
                const double q = th + lam * p;
                if (FIN) {
                    G.q[o + a] = q;
                } else {
                    G.x[o + a] += alpha * p;
                    r = G.r[o + a] - alpha * q;
                    G.r[o + a] = r;
                    rsh[a] = r;
                }
            }
            if (!FIN) {
                __syncthreads();
                if (a < dim) {
                    const double *Mh = h < G.Q ? G.Mh + 36 * (int64_t)h + a * 6 : G.Mh + 36 * (int64_t)G.Q + (h - G.Q);
                    double z = 0.0;
                    for (int c = 0; c < dim; c++) z += Mh[c] * rsh[c];
                    G.zp[o + a] = make_double2(z, p);
                    tz[0][a] = r * z;
                    tz[1][a] = r * r;
                }
                __syncthreads();
                if (threadIdx.x == 0 && !isnan(alpha))
                    for (int c = 0; c < dim; c++) { pq += tz[0][c]; rr2 += tz[1][c]; }
            }
        }
    } else {
        const int lb = row_block((int)blockIdx.x - G.m_nh, G.nrb);
        const int l = lb * 256 + (int)threadIdx.x;
        const bool on = l < G.nown;
        double q[3] = {0, 0, 0}, pr[3] = {0, 0, 0}, xo[3] = {0, 0, 0}, ro[3] = {0, 0, 0}, M[6] = {0, 0, 0, 0, 0, 0};
        int64_t o = 0;
        if (on) {
            o = G.hd + 3 * (int64_t)l;
#pragma unroll
            for (int c = 0; c < 3; c++) q[c] = G.q[o + c];
            // several pairs: the row's shares, then its cross slots (contiguous) — four at a time, their
            // loads issued before the first is added (the additions in the same order)
            if (G.tmulti) {
                const int ns = G.tnshare[l];
                for (int j0 = 1; j0 < ns; j0 += 4) {
                    double v[4][3];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int j = j0 + u < ns ? j0 + u : j0;
                        const double *s = G.qs + 3 * ((int64_t)(j - 1) * G.nown + l);
#pragma unroll
                        for (int c = 0; c < 3; c++) v[u][c] = s[c];
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        if (j0 + u < ns)
#pragma unroll
                            for (int c = 0; c < 3; c++) q[c] += v[u][c];
                }
            }
            {
                const int k0 = G.txoff[l], k1 = G.txoff[l + 1];
                for (int kb = k0; kb < k1; kb += 4) {
                    double v[4][3];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int64_t k = kb + u < k1 ? kb + u : kb;
#pragma unroll
                        for (int c = 0; c < 3; c++) v[u][c] = G.xc[3 * k + c];
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        if (kb + u < k1)
#pragma unroll
                            for (int c = 0; c < 3; c++) q[c] += v[u][c];
                }
            }
            if (FIN) {
#pragma unroll
                for (int c = 0; c < 3; c++) G.q[o + c] = q[c];
            } else {
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const double2 v = G.zp[o + c];
                    pr[c] = __fma_rn(beta, v.y, v.x);
                    xo[c] = G.x[o + c];
                    ro[c] = G.r[o + c];
                }
#pragma unroll
                for (int k = 0; k < 6; k++) M[k] = G.Mv[6 * (int64_t)l + k];
            }
        }
        if (!FIN && !own_alpha && !G.alpha_kernel) alpha = m2_alpha_wait(G, it);
        if (!FIN && on && !isnan(alpha)) {
            double r[3], z[3];
#pragma unroll
            for (int c = 0; c < 3; c++) {
                G.x[o + c] = xo[c] + alpha * pr[c];
                r[c] = ro[c] - alpha * q[c];
            }
            z[0] = M[0] * r[0] + M[1] * r[1] + M[3] * r[2];
            z[1] = M[1] * r[0] + M[2] * r[1] + M[4] * r[2];
            z[2] = M[3] * r[0] + M[4] * r[1] + M[5] * r[2];
#pragma unroll
            for (int c = 0; c < 3; c++) {
                G.r[o + c] = r[c];
                G.zp[o + c] = make_double2(z[c], pr[c]);
                pq += r[c] * z[c];
                rr2 += r[c] * r[c];
            }
        }
    }
    if (FIN) return;
    __shared__ double red[2][4];
    if (G.tparts && !last) {                       // the next k_sp_tile's workgroups sum them
        pair_tree(pq, rr2, red, G.m2part + 2 * blockIdx.x, 0);
        return;
    }
    pair_tree(pq, rr2, red, G.m2part + 2 * blockIdx.x, 1);
    m2_dots(G, it, red);
}

// sharded tile chain (G.sd && G.tile): the rank's share of the single-reduction record xb from the
// tile product's partials — per heavy vertex its sums of A z over the tiles (one workgroup each), z.Az
// from every tile workgroup's partial, (r.z, r.r) from the update's (or the setup's) row-block
// partials — as k_sp_phase2<MG 2>'s first workgroups form it from phase 1's; the host all-reduces xb
__global__ void __launch_bounds__(256) k_sp_txb(int it, const SpDev G) {
    __shared__ double red4[4];
    __shared__ double lds[256];
    (void)it;
    if (gated_off(G.gate) || G.rec[0] != 0.0) return;
    const int nh = G.Q + G.S, h = (int)blockIdx.x;
    if (h < nh) {
        const double t = tile_heavy_sum(G, h, lds);
        if ((int)threadIdx.x < (h < G.Q ? 6 : 1)) G.xb[3 + heavy_dof(G, h) + threadIdx.x] = t;
    } else if (h == nh) {
        double a = 0.0;
        for (int j = threadIdx.x; j < G.t_grid; j += 256) a += G.m1part[j];
        a = block_sum(a, red4);
        if (threadIdx.x == 0) G.xb[2] = a;
    } else {
        double a0 = 0.0, a1 = 0.0;
        for (int j = threadIdx.x; j <= G.nrb; j += 256) { a0 += G.upart[2 * j]; a1 += G.upart[2 * j + 1]; }
        a0 = block_sum(a0, red4);
        a1 = block_sum(a1, red4);
        if (threadIdx.x == 0) { G.xb[0] = a0; G.xb[1] = a1; }
    }
}


// halo exchange: rows' values (width doubles per row at base + width * row) into / out of a buffer
__global__ void k_sp_pack(int n, const int32_t *__restrict__ rows, int width, int64_t base, const double *__restrict__ src,
                          double *__restrict__ buf) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)n * width) return;
    const int64_t i = t / width, c = t % width;
    buf[t] = src[base + (int64_t)width * rows[i] + c];
}

__global__ void k_sp_unpack(int n, const int32_t *__restrict__ rows, int width, int64_t base, const double *__restrict__ buf,
                            double *__restrict__ dst) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)n * width) return;
    const int64_t i = t / width, c = t % width;
    dst[base + (int64_t)width * rows[i] + c] = buf[t];
}

// (z, p) = (v, 0): a vector the first CG iteration's product multiplies (p = z at it 0)
__global__ void k_sp_load_p(int64_t n, const double *__restrict__ v, double2 *__restrict__ zp) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t < n) zp[t] = make_double2(v[t], 0.0);
}

// problem order [heavy][points by id] <-> plan order [heavy][rows]
__global__ void k_sp_permute(int32_t P, int64_t hd, const int32_t *__restrict__ row_of_point, const double *__restrict__ src,
                             double *__restrict__ dst, int to_plan) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t < hd) { dst[t] = src[t]; return; }
    const int64_t u = t - hd;
    if (u >= 3 * (int64_t)P) return;
    const int64_t pt = u / 3, c = u % 3;
    const int64_t row = row_of_point[pt];
    if (to_plan) dst[hd + 3 * row + c] = src[hd + 3 * pt + c];
    else dst[hd + 3 * pt + c] = src[hd + 3 * row + c];
}

}  // namespace sp

static inline unsigned nblk(int64_t n, int bs) { return (unsigned)std::max<int64_t>((n + bs - 1) / bs, 1); }

#define SPL(NAME, KER, GRID, ...)                                          \
    do {                                                                   \
        if ((GRID) <= 0) break;                        /* (n = 0) */       \
        hipEvent_t e0_ = prof_begin(st);                                   \
        hipLaunchKernelGGL(KER, dim3(GRID), dim3(256), 0, st, __VA_ARGS__); \
        prof_end(NAME, e0_, (unsigned)(GRID), 0.0, st);                    \
    } while (0)

#define SPLS(NAME, KER, GRID, LDS, ...)                                              \
    do {                                                                             \
        if ((GRID) <= 0) break;                                                      \
        hipEvent_t e0_ = prof_begin(st);                                             \
        hipLaunchKernelGGL(KER, dim3(GRID), dim3(256), (size_t)(LDS), st, __VA_ARGS__); \
        prof_end(NAME, e0_, (unsigned)(GRID), 0.0, st);                              \
    } while (0)

template <class JT, int MG>
static void launch_phase2(const SpDev &G, int grid, int it, double lambda, const JT *pj, hipStream_t st) {
    if (G.p2u == 4) SPL("sp_phase2", (sp::k_sp_phase2<JT, MG, 4>), grid, it, G, lambda, pj);
    else if (G.p2u == 6) SPL("sp_phase2", (sp::k_sp_phase2<JT, MG, 6>), grid, it, G, lambda, pj);
    else SPL("sp_phase2", (sp::k_sp_phase2<JT, MG, 8>), grid, it, G, lambda, pj);
}

void sp_launch_glin(const SpDev &G, bool fp32, hipStream_t st) {
    if (G.glu == 4) {
        if (fp32) SPL("sp_glin_rows", (sp::k_sp_glin_rows<float, 4>), sp::row_grid(G.nrb2), G, G.pj32);
        else SPL("sp_glin_rows", (sp::k_sp_glin_rows<double, 4>), sp::row_grid(G.nrb2), G, G.pj);
    } else if (G.glu == 6) {
        if (fp32) SPL("sp_glin_rows", (sp::k_sp_glin_rows<float, 6>), sp::row_grid(G.nrb2), G, G.pj32);
        else SPL("sp_glin_rows", (sp::k_sp_glin_rows<double, 6>), sp::row_grid(G.nrb2), G, G.pj);
    } else {
        if (fp32) SPL("sp_glin_rows", (sp::k_sp_glin_rows<float, 8>), sp::row_grid(G.nrb2), G, G.pj32);
        else SPL("sp_glin_rows", (sp::k_sp_glin_rows<double, 8>), sp::row_grid(G.nrb2), G, G.pj);
    }
    if (G.nblk > 0) SPL("sp_glin_blocks", sp::k_sp_glin_blocks, G.nglb, G);
    if (G.nch > 0) SPL("sp_glin_heavy", sp::k_sp_glin_heavy, G.nch, G);
}

void sp_launch_maxdiag(const SpDev &G, double *out, hipStream_t st) {
    SPL("sp_maxdiag", sp::k_sp_maxdiag, 1, G, out, 0);
}

void sp_launch_maxdiag_heavy(const SpDev &G, double *out, hipStream_t st) {
    SPL("sp_maxdiag", sp::k_sp_maxdiag, 1, G, out, 1);
}

void sp_launch_cvt_j(const double *J, float *J32, int64_t n, hipStream_t st, const int *gate) {
    if (n > 0) SPL("sp_cvt_j", sp::k_sp_cvt_j, nblk(n, 256), J, J32, n, gate);
}

void sp_launch_setup(const SpDev &G, const double *rhs, double lambda, hipStream_t st) {
    const int grid = (G.nown + kSpUpdRows - 1) / kSpUpdRows + 1;
    hipEvent_t e0_ = prof_begin(st);
    hipLaunchKernelGGL(sp::k_sp_setup, dim3(grid), dim3(3 * kSpUpdRows), 0, st, G, rhs, lambda);
    prof_end("sp_setup", e0_, (unsigned)grid, 0.0, st);
}

void sp_launch_dots(const SpDev &G, int it, hipStream_t st) {
    SPL("sp_dots", sp::k_sp_dots, 1, it, G);
}

void sp_launch_product(const SpDev &G, int it, double lambda, bool fp32, hipStream_t st, bool last) {
    if (G.sd) {
        // sharded single-reduction chain: [m_nx heavy-z / row-term workgroups][phase-1 blocks];
        // [m_nh heavy-sum / scalar workgroups][row blocks]
        sp_launch_sd_phase1(G, it, lambda, fp32, st, nullptr, sp_merged_grid1(G));
        sp_launch_sd_phase2(G, it, lambda, fp32, st);
        return;
    }
    if (G.tile) {
        // [tiles, XCD-dealt][heavy dofs]; [m_nh heavy workgroups][row blocks]
        hipEvent_t e0_ = prof_begin(st);
        if (fp32) hipLaunchKernelGGL((sp::k_sp_tile<float>), dim3(G.t_grid), dim3(256), (size_t)G.tile_lds, st, it, G, G.Ja32, lambda);
        else hipLaunchKernelGGL((sp::k_sp_tile<double>), dim3(G.t_grid), dim3(256), (size_t)G.tile_lds, st, it, G, G.Ja, lambda);
        prof_end("sp_tile", e0_, (unsigned)G.t_grid, 0.0, st);
        if (G.alpha_kernel) SPL("sp_alpha", sp::k_sp_alpha, 1, it, G);
        SPL("sp_tupd", (sp::k_sp_tupd<0>), G.m_nh + sp::row_grid(G.nrb), it, G, lambda, last ? 1 : 0);
        return;
    }
    if (G.merged) {
        // [m_nx heavy-p / row-term workgroups][phase-1 blocks]; [m_nh heavy workgroups][row blocks]
        // (both extra counts multiples of 8, so the blocks keep their XCD)
        const int g1 = sp_merged_grid1(G), g2 = sp_merged_grid2(G);
        if (fp32) SPL("sp_phase1", (sp::k_sp_phase1<float, 1>), g1, it, G, G.Ja32, lambda);
        else SPL("sp_phase1", (sp::k_sp_phase1<double, 1>), g1, it, G, G.Ja, lambda);
        if (G.alpha_kernel) SPL("sp_alpha", sp::k_sp_alpha, 1, it, G);
        if (fp32) launch_phase2<float, 1>(G, g2, it, lambda, G.pj32, st);
        else launch_phase2<double, 1>(G, g2, it, lambda, G.pj, st);
        return;
    }
    if (G.nblk > 0) {
        if (fp32) SPL("sp_phase1", (sp::k_sp_phase1<float, 0>), G.nblk, it, G, G.Ja32, lambda);
        else SPL("sp_phase1", (sp::k_sp_phase1<double, 0>), G.nblk, it, G, G.Ja, lambda);
    }
    // one rank, G.fuse_heavy: + one workgroup per heavy vertex (its sums) before the row blocks
    const int grid = sp::row_grid(G.nrb2) + (G.fuse_heavy ? G.Q + G.S : 0);
    if (fp32) launch_phase2<float, 0>(G, grid, it, lambda, G.pj32, st);
    else launch_phase2<double, 0>(G, grid, it, lambda, G.pj, st);
}

void sp_launch_tile_sd(const SpDev &G, int it, double lambda, bool fp32, hipStream_t st, const int32_t *list, int n,
                       bool txb) {
    if (n > 0) {
        SpDev g = G;
        g.p1list = list;
        hipEvent_t e0_ = prof_begin(st);
        if (fp32) hipLaunchKernelGGL((sp::k_sp_tile<float, 1>), dim3(n), dim3(256), (size_t)G.tile_lds, st, it, g, G.Ja32, lambda);
        else hipLaunchKernelGGL((sp::k_sp_tile<double, 1>), dim3(n), dim3(256), (size_t)G.tile_lds, st, it, g, G.Ja, lambda);
        prof_end("sp_tile", e0_, (unsigned)n, 0.0, st);
    }
    if (txb) SPL("sp_txb", sp::k_sp_txb, G.Q + G.S + 2, it, G);
}

void sp_launch_tile_product(const SpDev &G, double lambda, bool fp32, hipStream_t st) {
    hipEvent_t e0_ = prof_begin(st);
    if (fp32) hipLaunchKernelGGL((sp::k_sp_tile<float>), dim3(G.t_grid), dim3(256), (size_t)G.tile_lds, st, 0, G, G.Ja32, lambda);
    else hipLaunchKernelGGL((sp::k_sp_tile<double>), dim3(G.t_grid), dim3(256), (size_t)G.tile_lds, st, 0, G, G.Ja, lambda);
    prof_end("sp_tile", e0_, (unsigned)G.t_grid, 0.0, st);
    SPL("sp_tupd", (sp::k_sp_tupd<1>), G.m_nh + sp::row_grid(G.nrb), 0, G, lambda, 1);
}

int sp_merged_grid1(const SpDev &G) { return 8 * ((G.nrb + 1 + 7) / 8) + G.nblk; }

void sp_launch_sd_phase1(const SpDev &G, int it, double lambda, bool fp32, hipStream_t st, const int32_t *list, int n) {
    SpDev g = G;
    g.p1list = list;
    if (fp32) SPL("sp_phase1", (sp::k_sp_phase1<float, 2>), n, it, g, G.Ja32, lambda);
    else SPL("sp_phase1", (sp::k_sp_phase1<double, 2>), n, it, g, G.Ja, lambda);
}

void sp_launch_sd_phase2(const SpDev &G, int it, double lambda, bool fp32, hipStream_t st) {
    const int g2 = G.m_nh + sp::row_grid(G.nrb2);
    if (fp32) launch_phase2<float, 2>(G, g2, it, lambda, G.pj32, st);
    else launch_phase2<double, 2>(G, g2, it, lambda, G.pj, st);
}
int sp_merged_grid2(const SpDev &G) { return 8 * ((G.Q + G.S + 7) / 8) + sp::row_grid(G.nrb2); }

void sp_launch_heavy(const SpDev &G, int it, double lambda, int stage, hipStream_t st) {
    // stage 1 over one workgroup per heavy vertex when the vertices have many blocks
    const int grid = (stage == 1 && G.heavy_split) ? G.Q + G.S + 1 : 1;
    SPL("sp_heavy", sp::k_sp_heavy, grid, it, G, lambda, stage);
}

void sp_launch_update_sd(const SpDev &G, int it, double lambda, int tail, hipStream_t st) {
    const int grid = (G.nown + kSpUpdRows - 1) / kSpUpdRows + 1;
    hipEvent_t e0_ = prof_begin(st);
    hipLaunchKernelGGL(sp::k_sp_update_sd, dim3(grid), dim3(3 * kSpUpdRows), 0, st, it, G, lambda, tail);
    prof_end("sp_update", e0_, (unsigned)grid, 0.0, st);
}

void sp_launch_update(const SpDev &G, int it, hipStream_t st) {
    const int grid = (G.nown + kSpUpdRows - 1) / kSpUpdRows + 1;
    hipEvent_t e0_ = prof_begin(st);
    hipLaunchKernelGGL(sp::k_sp_update, dim3(grid), dim3(3 * kSpUpdRows), 0, st, it, G);
    prof_end("sp_update", e0_, (unsigned)grid, 0.0, st);
}

void sp_launch_halo_pack(int n, const int32_t *rows, int width, int64_t base, const double *src, double *buf,
                         hipStream_t st) {
    if (n > 0) SPL("sp_halo_pack", sp::k_sp_pack, nblk((int64_t)n * width, 256), n, rows, width, base, src, buf);
}

void sp_launch_halo_unpack(int n, const int32_t *rows, int width, int64_t base, const double *buf, double *dst,
                           hipStream_t st) {
    if (n > 0) SPL("sp_halo_unpack", sp::k_sp_unpack, nblk((int64_t)n * width, 256), n, rows, width, base, buf, dst);
}

void sp_launch_load_p(int64_t n, const double *v, double2 *zp, hipStream_t st) {
    SPL("sp_load_p", sp::k_sp_load_p, nblk(n, 256), n, v, zp);
}

void sp_launch_permute_in(int32_t P, int64_t hd, const int32_t *row_of_point, const double *src, double *dst,
                          hipStream_t st) {
    SPL("sp_permute", sp::k_sp_permute, nblk(hd + 3 * (int64_t)P, 256), P, hd, row_of_point, src, dst, 1);
}

void sp_launch_permute_out(int32_t P, int64_t hd, const int32_t *row_of_point, const double *src, double *dst,
                           hipStream_t st) {
    SPL("sp_permute", sp::k_sp_permute, nblk(hd + 3 * (int64_t)P, 256), P, hd, row_of_point, src, dst, 0);
}

}  // namespace deftri
