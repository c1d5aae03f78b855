// Microbenchmark: sustained v_mfma_f64_16x16x4 and v_fma_f64 rates on one MI355X.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int CHAINS>
__global__ void __launch_bounds__(256) k_mfma(int iters, double *out) {
    dbl4 acc[CHAINS];
    for (int c = 0; c < CHAINS; c++) acc[c] = dbl4{0, 0, 0, 0};
    double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
    for (int i = 0; i < iters; i++)
#pragma unroll
        for (int c = 0; c < CHAINS; c++) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    double s = 0;
    for (int c = 0; c < CHAINS; c++) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    if (s == 12345.0) out[0] = s;
}

__global__ void __launch_bounds__(256) k_fma(int iters, double *out) {
    double x[8];
    for (int c = 0; c < 8; c++) x[c] = threadIdx.x * c * 1e-9;
    double a = 1.0000001, b = 1e-9;
    for (int i = 0; i < iters; i++)
#pragma unroll
        for (int c = 0; c < 8; c++) x[c] = fma(x[c], a, b);
    double s = 0;
    for (int c = 0; c < 8; c++) s += x[c];
    if (s == 12345.0) out[0] = s;
}

int main() {
    double *out;
    hipMalloc(&out, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    int grid = 256 * 8, iters = 4000;
    auto run = [&](const char *name, auto kern, double flop_per_iter_per_wave) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, 10, out);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, iters, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        double fl = flop_per_iter_per_wave * iters * grid * 4;
        printf("%-24s %8.3f ms  %7.2f TFLOP/s\n", name, ms, fl / (ms * 1e-3) / 1e12);
    };
    run("mfma_f64 chains=1", k_mfma<1>, 2048.0 * 1);
    run("mfma_f64 chains=2", k_mfma<2>, 2048.0 * 2);
    run("mfma_f64 chains=4", k_mfma<4>, 2048.0 * 4);
    run("mfma_f64 chains=8", k_mfma<8>, 2048.0 * 8);
    run("v_fma_f64 x8", k_fma, 64.0 * 2 * 8);
    return 0;
}
