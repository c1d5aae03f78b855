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

constexpr int DP = 65;   // padded LDS row (doubles) of the 64 x 64 diagonal block

// ------------------------------------------------------------------------------------------
// Blocked LDL^T + unit-lower inverse of one 64x64 panel diagonal block held in LDS (256 threads).
//   in : S[r][c] (c <= r) = A (rows/cols >= kb padded with the identity), S[c][r] (r > c) = 0
//   out: S[r][c] (c < r) = L, S[r][r] = D, S[c][r] (r > c) = X[r][c], X = L^{-1}
// Four 16-column sub-panels K, each: the 16x16 diagonal block's pivot chain in the registers of
// wave 0 (F), the inverse blocks of block row K and the sub-panel TRSM below it (B, f64 MFMA), the
// trailing Schur update and the inverse accumulators (U, f64 MFMA tiles).  Critical-path design
// (bit-identical to the first, ds_bpermute-based version; 21.0 -> 18.4 us per panel in isolation):
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
// A[r][g + 4q], X[r][g + 4q], q = 0..3): right-looking steps over the block's 16 pivots.  Branch-free
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
// rows kb..nrows-1 (nrows <= 64) below the kb x kb pivot block carry the panel's next rows: the
// right-looking steps of the kb pivots turn them into L21 = A21 L11^{-T} D^{-1} (the TRSM of the
// tile's remaining rows); their own "pivots" are never taken (steps past kb are no-ops) and the
// trailing part they update is scratch
__device__ __forceinline__ void diag_block_v2(double (*S)[DP], int kb, int nrows, int *flag) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int nsub = (max(kb, nrows) + 15) >> 4;
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

// panel k0 of front F (m rows, s own columns): the kb x kb diagonal block's LDL^T + inverse; with
// tail_rows (the fused-TRSM plan) also the TRSM of the remaining rows of the 64-row diagonal tile
// (rows k0+kb .. min(m, k0+64)), so the row tiles start at k0+64.  Without it (measured faster:
// partial panels then need only nsub sub-panels) k_trsm solves rows k0+kb..
// from_lds: the caller (k_update's diagonal-tile workgroup) already holds the block in S — lower
// kb x kb triangle, zero upper triangle, identity padding — so it skips the global round trip
__device__ __forceinline__ void diag_panel_v2(double *F, int m, int s, int k0, double *Li, double (*S)[DP], int *flag,
                                              bool tail_rows, bool from_lds = false) {
    const int kb = min(64, s - k0), mt = tail_rows ? min(64, m - k0) : kb;
    T2MARK(0);
    if (!from_lds) {
        double v[16];
#pragma unroll
        for (int q = 0; q < 16; q++) {
            int idx = threadIdx.x + 256 * q, c = idx >> 6, r = idx & 63;
            v[q] = (r < mt && c < kb && r >= c) ? F[(int64_t)(k0 + c) * m + k0 + r] : ((r == c && r >= kb) ? 1.0 : 0.0);
        }
#pragma unroll
        for (int q = 0; q < 16; q++) {
            int idx = threadIdx.x + 256 * q, c = idx >> 6, r = idx & 63;
            S[r][c] = v[q];
        }
    }
    __syncthreads();
    diag_block_v2(S, kb, mt, flag);
#pragma unroll
    for (int q = 0; q < 16; q++) {
        int idx = threadIdx.x + 256 * q, c = idx >> 6, r = idx & 63;
        if (r < mt && c < kb && r >= c) F[(int64_t)(k0 + c) * m + k0 + r] = S[r][c];
        if (r < kb && c < kb) Li[(int64_t)c * kb + r] = (r > c) ? S[c][r] : (r == c ? 1.0 : 0.0);
    }
#ifdef DEFTRI_DIAG_T2
    __syncthreads();
    T2MARK(41);
#endif
}

}  // namespace dev
}  // namespace deftri
