// diag_panel.h — 64x64 panel LDL^T + unit-lower inverse of the multifrontal factorization
// (the pivot chain of every panel step; included by kernels.hip and tools/micro/diag_bench.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

namespace deftri {
namespace dev {

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef double dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ double readlane_d(double v, int lane) {
    int2 p = __builtin_bit_cast(int2, v);
    p.x = __builtin_amdgcn_readlane(p.x, lane);
    p.y = __builtin_amdgcn_readlane(p.y, lane);
    return __builtin_bit_cast(double, p);
}

// 1/d from v_rcp_f64 and two Newton steps (≈0.5 ulp for the normal, positive pivots of an SPD
// block): a fraction of the latency of the IEEE division sequence on the 64-step pivot chain
__device__ __forceinline__ double rcp_d(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    return fma(r, e, r);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Blocked LDL^T + unit-lower inverse of one 64x64 panel diagonal block held in LDS (256 threads).
//   in : S[r][c] (c <= r) = A (rows/cols >= kb padded with the identity), S[c][r] (r > c) = 0
//   out: S[r][c] (c < r) = L, S[r][r] = D, S[c][r] (r > c) = X[r][c], X = L^{-1}
// Four 16-column sub-panels K.  Per sub-panel:
//   F  the 16x16 diagonal block and its inverse in the registers of wave 0: 16 right-looking
//      steps with cross-lane broadcasts, no barrier (A[r][c] -= l_r a_c, X[r][c] -= l_r X[j][c]);
//   X  (waves nrt..) finishes the inverse blocks of block row K: X_KJ = -X_KK T_KJ, J < K;
//   TR (waves 0..nrt-1) the sub-panel TRSM below it: L_IK = A_IK X_KK^T D_K^{-1};
//   U  the trailing Schur update on the lower triangle and the inverse accumulators
//      T_IJ += L_IK X_KJ (I > K, J <= K), all 16x16x16 f64 MFMA tiles.
// T_IJ accumulates in place in the upper-triangle slot of X_IJ (zero on entry).
constexpr int DP = 65;
__device__ __forceinline__ void diag_block(double (*S)[DP], int kb, int *flag) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    // rows/cols >= kb are identity padding: sub-blocks past nsub and pivot steps past kb are no-ops
    const int nsub = (kb + 15) >> 4;
#ifdef DEFTRI_DIAG_TIMING
    long long tp[16]; int ntp = 0;
    tp[ntp++] = clock64();
#endif
    for (int K = 0; K < nsub; K++) {
        const int j0 = 16 * K;
        const int jend = min(16, kb - j0);
        // ---- F: factor the diagonal block + its inverse in the registers of wave 0 (no barrier on
        //      the pivot chain).  Lane (r, g) = (lane & 15, lane >> 4) holds A[r][c] and X[r][c]
        //      for c = g, g+4, g+8, g+12 (both triangles of A, so row j is A[j][c] in lanes
        //      (j, g)); right-looking step j: d = A[j][j] (readlane), l_r = A[r][j] / d,
        //      A[r][c] -= l_r A[j][c] (r, c > j), X[r][c] -= l_r X[j][c] (r > j >= c).
        if (wv == 0) {
            const int r = lane & 15, g = lane >> 4, rowbase = lane & 48;
            double a[4], x[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int c = g + 4 * q;
                a[q] = (c <= r) ? S[j0 + r][j0 + c] : S[j0 + c][j0 + r];
                x[q] = (c == r) ? 1.0 : 0.0;
            }
#pragma unroll
            for (int j = 0; j < 16; j++) {
                if (j < jend) {
                    const double d = readlane_d(a[j >> 2], j + 16 * (j & 3));          // A[j][j]
                    const double arj = __shfl(a[j >> 2], r + 16 * (j & 3));            // A[r][j]
                    double ajc[4], xjc[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        ajc[q] = __shfl(a[q], rowbase | j);                            // A[j][c_q]
                        xjc[q] = __shfl(x[q], rowbase | j);                            // X[j][c_q]
                    }
                    const double lr = arj * rcp_d(d);
                    if (r > j) {
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const int c = g + 4 * q;
                            if (c > j) a[q] -= lr * ajc[q];
                            else x[q] -= lr * xjc[q];
                            if (c == j) a[q] = lr;                                     // L[r][j]
                        }
                    }
                    if (lane == 0 && d == 0.0) atomicOr(flag, 1);
                }
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int c = g + 4 * q;
                if (c <= r) S[j0 + r][j0 + c] = a[q];                                  // L (c < r), D (c == r)
                if (c < r) S[j0 + c][j0 + r] = x[q];                                   // X[r][c]
            }
        }
        __syncthreads();
#ifdef DEFTRI_DIAG_TIMING
        tp[ntp++] = clock64();
#endif
        const int nrt = nsub - 1 - K;                          // 16-row tiles below the sub-panel
        // ---- X: X_KJ = -X_KK T_KJ for J < K (T_KJ at S[16J + c][j0 + r]) ----
        if (wv >= nrt && wv - nrt < K) {
            const int J = wv - nrt, cidx = 16 * J + li;
            dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k4 = 0; k4 < 16; k4 += 4) {
                const int k = k4 + lk;
                const double av = (k == li) ? 1.0 : (k < li ? S[j0 + k][j0 + li] : 0.0);  // X_KK[li][k]
                const double bv = S[cidx][j0 + k];                                        // T_KJ[k][li]
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
            }
#pragma unroll
            for (int g = 0; g < 4; g++) S[cidx][j0 + lk + 4 * g] = -acc[g];             // X[j0+r][cidx]
        }
        // ---- TR: L[r][c] = sum_k A[r][j0+k] X[c][k] / d_c, one row tile per wave ----
        if (wv < nrt) {
            const int R = j0 + 16 + 16 * wv, c = j0 + li;
            const double rdc = 1.0 / S[c][c];
            dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k4 = 0; k4 < 16; k4 += 4) {
                const int k = k4 + lk;
                const double av = S[R + li][j0 + k];
                const double wk = ((k < li) ? S[j0 + k][c] : (k == li ? 1.0 : 0.0)) * rdc;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, wk, acc, 0, 0, 0);
            }
#pragma unroll
            for (int g = 0; g < 4; g++) S[R + lk + 4 * g][c] = acc[g];
        }
        if (K == nsub - 1) break;
        __syncthreads();
#ifdef DEFTRI_DIAG_TIMING
        tp[ntp++] = clock64();
#endif
        // ---- U: Schur tiles (Rt >= Ct) then inverse accumulators (I > K, J <= K) ----
        const int nsch = nrt * (nrt + 1) / 2, ninv = nrt * (K + 1);
        for (int t = wv; t < nsch + ninv; t += 4) {
            dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
            if (t < nsch) {
                int Rt = 0, Ct = t;
                while (Ct > Rt) { Ct -= Rt + 1; Rt++; }
                const int R = j0 + 16 + 16 * Rt, C = j0 + 16 + 16 * Ct;
#pragma unroll
                for (int k4 = 0; k4 < 16; k4 += 4) {
                    const int k = j0 + k4 + lk;
                    const double av = S[R + li][k] * S[k][k];
                    const double bv = S[C + li][k];
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
                }
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const int r = R + lk + 4 * g, c = C + li;
                    if (r >= c) S[r][c] -= acc[g];
                }
            } else {
                const int q = t - nsch, I = K + 1 + q / (K + 1), J = q % (K + 1);
                const int cidx = 16 * J + li;
#pragma unroll
                for (int k4 = 0; k4 < 16; k4 += 4) {
                    const int k = k4 + lk, kk = j0 + k;
                    const double av = S[16 * I + li][kk];                                 // L[16I+li][kk]
                    double bv;                                                            // X[kk][cidx]
                    if (J < K) bv = S[cidx][kk];
                    else bv = (k == li) ? 1.0 : (k > li ? S[cidx][kk] : 0.0);
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
                }
#pragma unroll
                for (int g = 0; g < 4; g++) S[cidx][16 * I + lk + 4 * g] += acc[g];       // T_IJ[r][c]
            }
        }
        __syncthreads();
#ifdef DEFTRI_DIAG_TIMING
        tp[ntp++] = clock64();
#endif
    }
    __syncthreads();
#ifdef DEFTRI_DIAG_TIMING
    tp[ntp++] = clock64();
    if (threadIdx.x == 0 && (blockIdx.x & 1023) == 0) {
        long long d[13];
        for (int q = 0; q < 13; q++) d[q] = (q + 1 < ntp) ? tp[q + 1] - tp[q] : 0;
        printf("[diagphase] kb %d: %lld %lld %lld | %lld %lld %lld | %lld %lld %lld | %lld %lld %lld | %lld\n", kb, d[0],
               d[1], d[2], d[3], d[4], d[5], d[6], d[7], d[8], d[9], d[10], d[11], d[12]);
    }
#endif
}

// load the panel diagonal block of (front F, panel k0) into S (identity padding), factor, store L/D
// into the front and Linv (kb x kb, column-major) into the inverse arena
__device__ __forceinline__ void diag_panel(double *F, int m, int s, int k0, double *Li, double (*S)[DP], int *flag) {
    const int kb = min(64, s - k0);
#ifdef DEFTRI_DIAG_TIMING
    long long tm0 = clock64();
#endif
    // all 16 loads per thread in flight at once (unrolled), then the LDS stores
    double v[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        int idx = threadIdx.x + 256 * q, c = idx >> 6, r = idx & 63;
        v[q] = (r < kb && c < kb && r >= c) ? F[(int64_t)(k0 + c) * m + k0 + r] : ((r == c && r >= kb) ? 1.0 : 0.0);
    }
#pragma unroll
    for (int q = 0; q < 16; q++) {
        int idx = threadIdx.x + 256 * q, c = idx >> 6, r = idx & 63;
        S[r][c] = v[q];
    }
    __syncthreads();
#ifdef DEFTRI_DIAG_TIMING
    long long tm1 = clock64();
#endif
    diag_block(S, kb, flag);
#ifdef DEFTRI_DIAG_TIMING
    long long tm2 = clock64();
#endif
#pragma unroll
    for (int q = 0; q < 16; q++) {
        int idx = threadIdx.x + 256 * q, c = idx >> 6, r = idx & 63;
        if (r < kb && c < kb) {
            if (r >= c) F[(int64_t)(k0 + c) * m + k0 + r] = S[r][c];
            Li[(int64_t)c * kb + r] = (r > c) ? S[c][r] : (r == c ? 1.0 : 0.0);
        }
    }
#ifdef DEFTRI_DIAG_TIMING
    __syncthreads();
    long long tm3 = clock64();
    if (threadIdx.x == 0 && (blockIdx.x & 1023) == 0)
        printf("[diagtime] blk %d load %lld block %lld store %lld\n", (int)blockIdx.x, tm1 - tm0, tm2 - tm1, tm3 - tm2);
#endif
}

// ------------------------------------------------------------------------------------------
// v2: the same arithmetic (bit-identical L, D, X), shorter critical path
//   * the 16-step pivot chain broadcasts through DPP / permlane instead of ds_bpermute: row j of
//     the block (same 16-lane DPP row) by v_mov_b64_dpp row_newbcast:j, column j (one lane per
//     row, in DPP row j&3) by v_permlane16_swap + v_permlane32_swap;
//   * one-step lookahead: wave 0 finishes the Schur tile (K+1, K+1) of sub-panel K itself and goes
//     straight on to the pivot chain of K+1 while waves 1-3 apply the rest of sub-panel K's update
//     (Schur tiles and inverse accumulators): two barriers per sub-panel instead of three, and the
//     bulk of the MFMA update off the chain;
// ------------------------------------------------------------------------------------------
template <int N, int I = 0, typename Fn>
__device__ __forceinline__ void static_for(Fn &&fn) {
    if constexpr (I < N) {
        fn(std::integral_constant<int, I>{});
        static_for<N, I + 1>(fn);
    }
}

// lane l of every 16-lane row <- lane J of that row
template <int J>
__device__ __forceinline__ double bcast_in_row(double v) {
    long long b = __builtin_bit_cast(long long, v);
    b = __builtin_amdgcn_update_dpp(0LL, b, 0x150 + J, 0xf, 0xf, true);    // row_newbcast:J (all lanes written)
    return __builtin_bit_cast(double, b);
}

// every row <- row R (lane l <- lane 16R + (l & 15))
template <int R>
__device__ __forceinline__ double bcast_row(double v) {
    int2 p = __builtin_bit_cast(int2, v);
    // permlane16_swap(v, v): [0] = rows (0,0,2,2), [1] = rows (1,1,3,3)
    auto lo16 = __builtin_amdgcn_permlane16_swap((unsigned)p.x, (unsigned)p.x, false, false);
    auto hi16 = __builtin_amdgcn_permlane16_swap((unsigned)p.y, (unsigned)p.y, false, false);
    const unsigned tlo = lo16[R & 1], thi = hi16[R & 1];
    // permlane32_swap(t, t): [0] = rows (0,1,0,1) of t, [1] = rows (2,3,2,3)
    auto lo32 = __builtin_amdgcn_permlane32_swap(tlo, tlo, false, false);
    auto hi32 = __builtin_amdgcn_permlane32_swap(thi, thi, false, false);
    p.x = (int)lo32[R >> 1];
    p.y = (int)hi32[R >> 1];
    return __builtin_bit_cast(double, p);
}

// pivot chain of one 16x16 diagonal block in the registers of one wave (lane = r + 16 g holds
// A[r][g + 4q], X[r][g + 4q], q = 0..3); same operations as diag_block's F phase.  Branch-free
// steps (selects), the zero-pivot test folded into one flag write at the end.
template <bool FULL>
__device__ __forceinline__ void f_chain(double (*S)[DP], int j0, int jend, int *flag) {
    const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
    double a[4], x[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int c = g + 4 * q;
        a[q] = (c <= r) ? S[j0 + r][j0 + c] : S[j0 + c][j0 + r];
        x[q] = (c == r) ? 1.0 : 0.0;
    }
    bool zp = false;
    static_for<16>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        if (FULL || J < jend) {
            const double d = readlane_d(a[J >> 2], J + 16 * (J & 3));           // A[J][J]
            const double arj = bcast_row<J & 3>(a[J >> 2]);                      // A[r][J]
            double ajc[4], xjc[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                ajc[q] = (4 * q + 3 > J) ? bcast_in_row<J>(a[q]) : 0.0;          // A[J][c_q]
                xjc[q] = (4 * q <= J) ? bcast_in_row<J>(x[q]) : 0.0;             // X[J][c_q]
            }
            const double lr = arj * rcp_d(d);
            const bool below = r > J;
            const double lrb = below ? lr : 0.0;           // rows r <= J are final: fma(-0, v, a) == a
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int c = g + 4 * q;
                if (4 * q > J) {
                    a[q] = fma(-lrb, ajc[q], a[q]);                                 // every c > J
                } else if (4 * q + 3 >= J) {                                        // q == J >> 2: mixed
                    const double an = fma(-lr, ajc[q], a[q]);
                    a[q] = (below && c > J) ? an : ((below && c == J) ? lr : a[q]);  // L[r][J] at c == J
                }
                if (4 * q + 3 <= J) {
                    x[q] = fma(-lrb, xjc[q], x[q]);                                 // every c <= J
                } else if (4 * q <= J) {
                    const double xn = fma(-lr, xjc[q], x[q]);
                    x[q] = (below && c <= J) ? xn : x[q];
                }
            }
            zp |= (d == 0.0);
        }
    });
    if (zp && lane == 0) atomicOr(flag, 1);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int c = g + 4 * q;
        if (c <= r) S[j0 + r][j0 + c] = a[q];                                    // L (c < r), D (c == r)
        if (c < r) S[j0 + c][j0 + r] = x[q];                                     // X[r][c]
    }
}

// one task of sub-panel K's update U_K (nrt = row tiles below it): t < nrt(nrt+1)/2 is the Schur
// tile (Rt >= Ct) A_RC -= L_RK D_K L_CK^T, otherwise the inverse accumulator T_IJ += L_IK X_KJ
// (I > K, J <= K).  Operands for the 4 k-steps are read into av/bv; apply writes the result.
struct UTask { int kind, R, C, I, J; };
__device__ __forceinline__ UTask u_task(int K, int nrt, int t) {
    const int nsch = nrt * (nrt + 1) / 2;
    const int j0 = 16 * K;
    UTask u;
    if (t < nsch) {
        int Rt = 0, Ct = t;
        while (Ct > Rt) { Ct -= Rt + 1; Rt++; }
        u.kind = 0; u.R = j0 + 16 + 16 * Rt; u.C = j0 + 16 + 16 * Ct; u.I = u.J = 0;
    } else {
        const int q = t - nsch;
        u.kind = 1; u.I = K + 1 + q / (K + 1); u.J = q % (K + 1); u.R = u.C = 0;
    }
    return u;
}
__device__ __forceinline__ void u_operands(double (*S)[DP], int K, const UTask &u, double av[4], double bv[4]) {
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4, j0 = 16 * K;
    if (u.kind == 0) {
#pragma unroll
        for (int k4 = 0; k4 < 4; k4++) {
            const int k = j0 + 4 * k4 + lk;
            av[k4] = S[u.R + li][k] * S[k][k];
            bv[k4] = S[u.C + li][k];
        }
    } else {
        const int cidx = 16 * u.J + li;
#pragma unroll
        for (int k4 = 0; k4 < 4; k4++) {
            const int k = 4 * k4 + lk, kk = j0 + k;
            av[k4] = S[16 * u.I + li][kk];                                       // L[16I+li][kk]
            if (u.J < K) bv[k4] = S[cidx][kk];                                   // X[kk][cidx]
            else bv[k4] = (k == li) ? 1.0 : (k > li ? S[cidx][kk] : 0.0);
        }
    }
}
__device__ __forceinline__ void u_apply(double (*S)[DP], const UTask &u, const dbl4 &acc) {
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
    if (u.kind == 0) {
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const int r = u.R + lk + 4 * g, c = u.C + li;
            if (r >= c) S[r][c] -= acc[g];
        }
    } else {
        const int cidx = 16 * u.J + li;
#pragma unroll
        for (int g = 0; g < 4; g++) S[cidx][16 * u.I + lk + 4 * g] += acc[g];            // T_IJ[r][c]
    }
}
// up to NT tasks of one wave, their MFMA chains interleaved
template <int NT>
__device__ __forceinline__ void u_tasks(double (*S)[DP], int K, int nrt, const int *ts, int n) {
    UTask u[NT];
    double av[NT][4], bv[NT][4];
    dbl4 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; i++) {
        acc[i] = dbl4{0.0, 0.0, 0.0, 0.0};
        if (i < n) { u[i] = u_task(K, nrt, ts[i]); u_operands(S, K, u[i], av[i], bv[i]); }
    }
#pragma unroll
    for (int k4 = 0; k4 < 4; k4++)
#pragma unroll
        for (int i = 0; i < NT; i++)
            if (i < n) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i][k4], bv[i][k4], acc[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < NT; i++)
        if (i < n) u_apply(S, u[i], acc[i]);
}

#ifdef DEFTRI_DIAG_T2
__device__ long long g_diag_t2[64];
#define T2MARK(i) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_diag_t2[i] = wall_clock64(); } while (0)
#define T2MARKW(i, w) do { if (threadIdx.x == 64 * (w) && blockIdx.x == 0) g_diag_t2[i] = wall_clock64(); } while (0)
#else
#define T2MARK(i) do {} while (0)
#define T2MARKW(i, w) do {} while (0)
#endif
__device__ __forceinline__ void diag_block_v2(double (*S)[DP], int kb, int *flag) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int nsub = (kb + 15) >> 4;
    T2MARK(1);
    for (int K = 0; K < nsub; K++) {
        const int j0 = 16 * K;
        // ---- A_K: wave 0 runs the pivot chain of block K (its tile (K, K) is final: wave 0 applied
        //      sub-panel K-1's update to it at the end of the previous step); waves 1-3 apply the
        //      rest of sub-panel K-1's update (Schur tiles t >= 1 and the inverse accumulators) ----
        if (wv == 0) {
            if (kb - j0 >= 16) f_chain<true>(S, j0, 16, flag);
            else f_chain<false>(S, j0, kb - j0, flag);
            T2MARK(2 + 8 * K);
        } else if (K > 0) {
            const int Kp = K - 1, nrtp = nsub - 1 - Kp;
            const int ntask = nrtp * (nrtp + 1) / 2 + nrtp * (Kp + 1);
            int ts[3], n = 0;
            for (int t = wv; t < ntask; t += 3) ts[n++] = t;                    // t = 0 was wave 0's
            for (int i = 0; i < n; i++) u_tasks<1>(S, Kp, nrtp, ts + i, 1);   // one at a time: fits 128 VGPRs
            T2MARKW(3 + 8 * K, 1);
        }
        __syncthreads();
        T2MARK(4 + 8 * K);
        const int nrt = nsub - 1 - K;
        // ---- B_K: X_KJ = -X_KK T_KJ (J < K) and the sub-panel TRSM L_IK = A_IK X_KK^T D_K^{-1} ----
        if (wv >= nrt && wv - nrt < K) {
            const int J = wv - nrt, cidx = 16 * J + li;
            dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k4 = 0; k4 < 16; k4 += 4) {
                const int k = k4 + lk;
                const double av = (k == li) ? 1.0 : (k < li ? S[j0 + k][j0 + li] : 0.0);  // X_KK[li][k]
                const double bv = S[cidx][j0 + k];                                        // T_KJ[k][li]
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
            }
#pragma unroll
            for (int g = 0; g < 4; g++) S[cidx][j0 + lk + 4 * g] = -acc[g];             // X[j0+r][cidx]
        }
        if (wv < nrt) {
            const int R = j0 + 16 + 16 * wv, c = j0 + li;
            const double rdc = 1.0 / S[c][c];
            dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k4 = 0; k4 < 16; k4 += 4) {
                const int k = k4 + lk;
                const double av = S[R + li][j0 + k];
                const double wk = ((k < li) ? S[j0 + k][c] : (k == li ? 1.0 : 0.0)) * rdc;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, wk, acc, 0, 0, 0);
            }
#pragma unroll
            for (int g = 0; g < 4; g++) S[R + lk + 4 * g][c] = acc[g];
        }
        T2MARK(5 + 8 * K);
        if (K == nsub - 1) break;
        __syncthreads();
        T2MARK(6 + 8 * K);
        // ---- C_K: wave 0 applies sub-panel K's update to tile (K+1, K+1) (task 0) and moves on
        //      to the next pivot chain; the other tiles are left to waves 1-3 in A_{K+1} ----
        if (wv == 0) {
            const int t0 = 0;
            u_tasks<1>(S, K, nrt, &t0, 1);
            wave_sync();
            T2MARK(7 + 8 * K);
        }
    }
    __syncthreads();
    T2MARK(40);
}

__device__ __forceinline__ void diag_panel_v2(double *F, int m, int s, int k0, double *Li, double (*S)[DP], int *flag) {
    const int kb = min(64, s - k0);
    T2MARK(0);
    double v[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        int idx = threadIdx.x + 256 * q, c = idx >> 6, r = idx & 63;
        v[q] = (r < kb && c < kb && r >= c) ? F[(int64_t)(k0 + c) * m + k0 + r] : ((r == c && r >= kb) ? 1.0 : 0.0);
    }
#pragma unroll
    for (int q = 0; q < 16; q++) {
        int idx = threadIdx.x + 256 * q, c = idx >> 6, r = idx & 63;
        S[r][c] = v[q];
    }
    __syncthreads();
    diag_block_v2(S, kb, flag);
#pragma unroll
    for (int q = 0; q < 16; q++) {
        int idx = threadIdx.x + 256 * q, c = idx >> 6, r = idx & 63;
        if (r < kb && c < kb) {
            if (r >= c) F[(int64_t)(k0 + c) * m + k0 + r] = S[r][c];
            Li[(int64_t)c * kb + r] = (r > c) ? S[c][r] : (r == c ? 1.0 : 0.0);
        }
    }
#ifdef DEFTRI_DIAG_T2
    __syncthreads();
    T2MARK(41);
#endif
}

}  // namespace dev
}  // namespace deftri
