// Microbenchmark: the multifrontal trailing update C -= L D L^T (k_update's K loop) on synthetic
// fronts — the current register-streaming kernel (A) against an LDS-staged variant (B) in which the
// workgroup loads each k-chunk of both operand panels once (16-byte loads, d folded in at staging)
// and the waves read their MFMA fragments from LDS.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 upd_bench.hip -o upd_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef double dbl2 __attribute__((ext_vector_type(2)));

#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ int xcd_task(int ntask) {
    int per = (ntask + 7) >> 3;
    return (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
}

// ---- A: the production kernel's loop (operands straight from global, 2-stage prefetch) ----
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
k_updA(int ntask, const int *__restrict__ tasks, int kA, int K, int m, double *__restrict__ arena) {
    int t = xcd_task(ntask);
    if (t >= ntask) return;
    int f = tasks[3 * t], ti = tasks[3 * t + 1], tj = tasks[3 * t + 2];
    double *F = arena + (int64_t)f * m * m;
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int rb = ti + (w & 1) * 32, cb = tj + (w >> 1) * 32;
    int kl = lane >> 4, il = lane & 15;
    double cv[2][2][4];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                int c = cb + 16 * a + kl + 4 * g, r = rb + 16 * b + il;
                cv[a][b][g] = (c < m && r < m) ? F[(int64_t)c * m + r] : 0.0;
            }
    dbl4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
    const bool p0ok = cb + il < m, p1ok = cb + 16 + il < m, q0ok = rb + il < m, q1ok = rb + 16 + il < m;
    constexpr int PD = 2;
    double cd[PD], c0[PD], c1[PD], c2[PD], c3[PD], nd[PD], n0[PD], n1[PD], n2[PD], n3[PD];
    auto loadk = [&](int kb0, double *d, double *x0, double *x1, double *y0, double *y1) {
#pragma unroll
        for (int u = 0; u < PD; u++) {
            int kk = kb0 + 4 * u + kl;
            bool ok = kk < K;
            const double *col = F + (int64_t)(kA + kk) * m;
            d[u] = ok ? col[kA + kk] : 0.0;
            x0[u] = (ok && p0ok) ? col[cb + il] : 0.0;
            x1[u] = (ok && p1ok) ? col[cb + 16 + il] : 0.0;
            y0[u] = (ok && q0ok) ? col[rb + il] : 0.0;
            y1[u] = (ok && q1ok) ? col[rb + 16 + il] : 0.0;
        }
    };
    loadk(0, cd, c0, c1, c2, c3);
    for (int kb0 = 0; kb0 < K; kb0 += 4 * PD) {
        const bool more = kb0 + 4 * PD < K;
        if (more) loadk(kb0 + 4 * PD, nd, n0, n1, n2, n3);
#pragma unroll
        for (int u = 0; u < PD; u++) {
            double p0 = c0[u] * cd[u], p1 = c1[u] * cd[u];
            acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0, c2[u], acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0, c3[u], acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1, c2[u], acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1, c3[u], acc[1][1], 0, 0, 0);
        }
        if (more)
#pragma unroll
            for (int u = 0; u < PD; u++) { cd[u] = nd[u]; c0[u] = n0[u]; c1[u] = n1[u]; c2[u] = n2[u]; c3[u] = n3[u]; }
    }
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                int c = cb + 16 * a + kl + 4 * g, r = rb + 16 * b + il;
                if (c < m && r < m) F[(int64_t)c * m + r] = cv[a][b][g] - acc[a][b][g];
            }
}

// ---- B: LDS-staged operands.  Chunk = KC k-columns; thread t stages column k = t / 16 of the
// chunk, rows 4 (t % 16) .. +3 of both 64-row operand panels (two 16-byte loads each); P = L_c d_k
// is scaled once at staging.  Double-buffered: chunk c+1's loads are in flight while chunk c's MFMAs
// run; one barrier per chunk. ----
constexpr int LQ = 64 + 4;   // padded row length (doubles) of one staged k-column
template <int KC, int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
k_updB(int ntask, const int *__restrict__ tasks, int kA, int K, int m, double *__restrict__ arena) {
    static_assert(KC == 16 || KC == 32, "KC");
    __shared__ double Ps[2][KC][LQ], Qs[2][KC][LQ];
    int t = xcd_task(ntask);
    if (t >= ntask) return;
    int f = tasks[3 * t], ti = tasks[3 * t + 1], tj = tasks[3 * t + 2];
    double *F = arena + (int64_t)f * m * m;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int rb = (w & 1) * 32, cb = (w >> 1) * 32;   // quadrant inside the tile
    const int kl = lane >> 4, il = lane & 15;
    // staging role
    constexpr int NV = KC / 8;                       // dbl2 per panel per thread
    const int sk = tid / (256 / KC), sr = (tid % (256 / KC)) * (2 * NV);
    dbl2 pv[NV], qv[NV];
    double dv;
    auto stage_load = [&](int c0) {
        const int kk = c0 + sk;
        const bool ok = kk < K;
        const double *col = F + (int64_t)(kA + kk) * m;
        dv = ok ? col[kA + kk] : 0.0;
#pragma unroll
        for (int v = 0; v < NV; v++) {
            pv[v] = (ok && tj + sr + 2 * v < m) ? *(const dbl2 *)(col + tj + sr + 2 * v) : dbl2{0.0, 0.0};
            qv[v] = (ok && ti + sr + 2 * v < m) ? *(const dbl2 *)(col + ti + sr + 2 * v) : dbl2{0.0, 0.0};
        }
    };
    auto stage_store = [&](int buf) {
#pragma unroll
        for (int v = 0; v < NV; v++) {
            *(dbl2 *)&Ps[buf][sk][sr + 2 * v] = pv[v] * dv;
            *(dbl2 *)&Qs[buf][sk][sr + 2 * v] = qv[v];
        }
    };
    stage_load(0);
    // C prefetch (this wave's quadrant)
    double cv[2][2][4];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                int c = tj + cb + 16 * a + kl + 4 * g, r = ti + rb + 16 * b + il;
                cv[a][b][g] = (c < m && r < m) ? F[(int64_t)c * m + r] : 0.0;
            }
    dbl4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
    stage_store(0);
    __syncthreads();
    const int nch = (K + KC - 1) / KC;
    for (int c = 0; c < nch; c++) {
        const int buf = c & 1;
        if (c + 1 < nch) stage_load((c + 1) * KC);
#pragma unroll
        for (int k4 = 0; k4 < KC; k4 += 4) {
            const double p0 = Ps[buf][k4 + kl][cb + il], p1 = Ps[buf][k4 + kl][cb + 16 + il];
            const double q0 = Qs[buf][k4 + kl][rb + il], q1 = Qs[buf][k4 + kl][rb + 16 + il];
            acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0, q0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0, q1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1, q0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1, q1, acc[1][1], 0, 0, 0);
        }
        if (c + 1 < nch) stage_store(buf ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                int c = tj + cb + 16 * a + kl + 4 * g, r = ti + rb + 16 * b + il;
                if (c < m && r < m) F[(int64_t)c * m + r] = cv[a][b][g] - acc[a][b][g];
            }
}

static void run_case(int nf, int m, int K, int VB) {
    std::vector<int> tasks;
    for (int f = 0; f < nf; f++)
        for (int tj = K; tj < m; tj += 64)
            for (int ti = tj; ti < m; ti += 64) { tasks.push_back(f); tasks.push_back(ti); tasks.push_back(tj); }
    const int nt = (int)tasks.size() / 3;
    double flops = 0;
    for (int q = 0; q < nt; q++) {
        int ti = tasks[3 * q + 1], tj = tasks[3 * q + 2];
        flops += 2.0 * std::min(64, m - ti) * std::min(64, m - tj) * K;
    }
    const size_t n = (size_t)nf * m * m;
    std::vector<double> h(n);
    srand(5);
    for (auto &x : h) x = rand() / (double)RAND_MAX - 0.5;
    double *dA, *dB; int *dt;
    HC(hipMalloc(&dA, n * 8)); HC(hipMalloc(&dB, n * 8)); HC(hipMalloc(&dt, tasks.size() * 4));
    auto kB = VB == 0 ? k_updB<16, 4> : VB == 1 ? k_updB<32, 2> : VB == 2 ? k_updB<16, 2> : k_updB<32, 4>;
    HC(hipMemcpy(dt, tasks.data(), tasks.size() * 4, hipMemcpyHostToDevice));
    HC(hipMemcpy(dA, h.data(), n * 8, hipMemcpyHostToDevice));
    HC(hipMemcpy(dB, h.data(), n * 8, hipMemcpyHostToDevice));
    const unsigned grid = 8 * ((nt + 7) / 8);
    hipLaunchKernelGGL(k_updA, dim3(grid), dim3(256), 0, 0, nt, dt, 0, K, m, dA);
    hipLaunchKernelGGL(kB, dim3(grid), dim3(256), 0, 0, nt, dt, 0, K, m, dB);
    HC(hipDeviceSynchronize());
    std::vector<double> a(n), b(n);
    HC(hipMemcpy(a.data(), dA, n * 8, hipMemcpyDeviceToHost));
    HC(hipMemcpy(b.data(), dB, n * 8, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < n; i++) bad += memcmp(&a[i], &b[i], 8) != 0;
    hipEvent_t e0, e1;
    HC(hipEventCreate(&e0)); HC(hipEventCreate(&e1));
    float msA = 0, msB = 0;
    const int reps = 20;
    for (int v = 0; v < 2; v++) {
        HC(hipEventRecord(e0));
        for (int r = 0; r < reps; r++) {
            if (v == 0) hipLaunchKernelGGL(k_updA, dim3(grid), dim3(256), 0, 0, nt, dt, 0, K, m, dA);
            else hipLaunchKernelGGL(kB, dim3(grid), dim3(256), 0, 0, nt, dt, 0, K, m, dB);
        }
        HC(hipEventRecord(e1));
        HC(hipEventSynchronize(e1));
        HC(hipEventElapsedTime(v == 0 ? &msA : &msB, e0, e1));
    }
    msA /= reps; msB /= reps;
    printf("B%d fronts %4d m %5d K %3d tiles %6d: A %8.1f us %6.2f TF/s | B %8.1f us %6.2f TF/s | %zu differ\n",
           VB, nf, m, K, nt, 1e3 * msA, flops / (msA * 1e-3) / 1e12, 1e3 * msB, flops / (msB * 1e-3) / 1e12, bad);
    HC(hipFree(dA)); HC(hipFree(dB)); HC(hipFree(dt));
}

int main() {
    for (int vb = 0; vb < 4; vb++) {
        run_case(1, 2048, 256, vb);
        run_case(11, 2000, 256, vb);
        run_case(34, 1300, 256, vb);
        run_case(129, 650, 162, vb);
        run_case(872, 290, 66, vb);
        run_case(6322, 170, 96, vb);
    }
    return 0;
}
