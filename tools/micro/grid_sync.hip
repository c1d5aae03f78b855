// Microbenchmark: cost of a grid-wide barrier on MI355X — cooperative-groups grid.sync() vs. a
// hand-rolled atomic-counter barrier (sense reversal, device-scope acquire/release).
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <cstdio>
namespace cg = cooperative_groups;
__global__ void k_cg(int *x, int n) {
    cg::grid_group g = cg::this_grid();
    for (int i = 0; i < n; i++) { if (blockIdx.x == 0 && threadIdx.x == 0) x[0]++; g.sync(); }
}
__device__ __forceinline__ void grid_barrier(unsigned *count, unsigned *gen, unsigned nblocks) {
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __atomic_thread_fence(__ATOMIC_RELEASE);
        unsigned arrived = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (arrived == nblocks - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g0) __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}
__global__ void k_atomic(int *x, int n, unsigned *count, unsigned *gen) {
    for (int i = 0; i < n; i++) {
        if (blockIdx.x == 0 && threadIdx.x == 0) x[0]++;
        grid_barrier(count, gen, gridDim.x);
    }
}
int main() {
    int *x; unsigned *cnt;
    hipMalloc(&x, 4); hipMemset(x, 0, 4);
    hipMalloc(&cnt, 8); hipMemset(cnt, 0, 8);
    int n = 1000;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int grid : {256, 512, 1024}) {
        void *args[] = {&x, &n};
        hipEventRecord(e0);
        hipError_t err = hipLaunchCooperativeKernel((const void *)k_cg, dim3(grid), dim3(256), args, 0, 0);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("cg     grid %4d err %d: %7.3f us per barrier\n", grid, (int)err, 1e3 * ms / n);
        unsigned *c = cnt, *g = cnt + 1;
        void *args2[] = {&x, &n, &c, &g};
        hipEventRecord(e0);
        err = hipLaunchCooperativeKernel((const void *)k_atomic, dim3(grid), dim3(256), args2, 0, 0);
        hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("atomic grid %4d err %d: %7.3f us per barrier\n", grid, (int)err, 1e3 * ms / n);
    }
    hipEventRecord(e0);
    for (int i = 0; i < 1000; i++) hipLaunchKernelGGL(k_cg, dim3(1), dim3(64), 0, 0, x, 0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("empty kernel launch back-to-back: %.3f us each\n", 1e3 * ms / 1000);
    int h; hipMemcpy(&h, x, 4, hipMemcpyDeviceToHost); printf("x %d\n", h);
}
