// Microbenchmark: do small kernels on different HIP streams overlap on MI355X?
// n streams each launch K kernels of G workgroups that spin ~T us; wall time vs 1 stream.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
__global__ void k_spin(long long cycles, int *out) {
    long long t0 = wall_clock64();
    while (wall_clock64() - t0 < cycles) {}
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}
__global__ void k_spin_scratch(long long cycles, int *out, int idx) {
    volatile double buf[16];
    for (int i = 0; i < 16; i++) buf[i] = i;
    long long t0 = wall_clock64();
    while (wall_clock64() - t0 < cycles) {}
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (int)buf[idx & 15];
}
__global__ void k_spin_lds(long long cycles, int *out) {
    __shared__ double S[64][65];
    S[threadIdx.x & 63][threadIdx.x >> 6] = 1.0;
    __syncthreads();
    long long t0 = wall_clock64();
    while (wall_clock64() - t0 < cycles) {}
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (int)S[3][2];
}
int main(int argc, char **argv) {
    int K = 400, G = 16;
    double us = 5.0;
    int *d; hipMalloc(&d, 64);
    int prio_lo = 0, prio_hi = 0;
    hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    std::vector<hipStream_t> st(8);
    for (auto &s : st) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    long long cyc = (long long)(us * 100);   // wall_clock64: 100 MHz
    int kind = argc > 1 ? atoi(argv[1]) : 0;
    for (int mode = 0; mode < 2; mode++)
    for (int ns : {1, 2, 3, 4, 8}) {
        hipDeviceSynchronize();
        auto t0 = std::chrono::steady_clock::now();
        if (mode == 0) {   // interleaved launch order
            for (int k = 0; k < K; k++)
                for (int s = 0; s < ns; s++) {
                    if (kind == 0) hipLaunchKernelGGL(k_spin, dim3(G), dim3(256), 0, st[s], cyc, d);
                    else if (kind == 1) hipLaunchKernelGGL(k_spin_scratch, dim3(G), dim3(256), 0, st[s], cyc, d, k);
                    else hipLaunchKernelGGL(k_spin_lds, dim3(G), dim3(256), 0, st[s], cyc, d);
                }
        } else {           // stream after stream (what a per-lane enqueue does)
            for (int s = 0; s < ns; s++)
                for (int k = 0; k < K; k++) {
                    if (kind == 0) hipLaunchKernelGGL(k_spin, dim3(G), dim3(256), 0, st[s], cyc, d);
                    else if (kind == 1) hipLaunchKernelGGL(k_spin_scratch, dim3(G), dim3(256), 0, st[s], cyc, d, k);
                    else hipLaunchKernelGGL(k_spin_lds, dim3(G), dim3(256), 0, st[s], cyc, d);
                }
        }
        hipDeviceSynchronize();
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::printf("kind %d mode %s streams %d: %d x %d launches of %.1f us: %.2f ms (%.2f us per launch per stream)\n", kind,
                    mode ? "blocked" : "interleaved", ns, ns, K, us, ms, 1e3 * ms / K);
    }
    return 0;
}
