// fetch_calib.hip — calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access widths the
// iterative plan's CG kernels use (MI355X_MICROARCH.md §HBM: "other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").  Each kernel streams a known byte
// count once, coalesced, at one width per lane: 4 B (float, the fp32-stored Jacobian columns), 8 B
// (double: the ARAP J columns, W, s_e, packed J slices), 16 B (double2: the (z, p) pairs), plus an
// 8-B indexed gather over a permutation (phase 2's s_e reads) and 8-B / 16-B streaming stores.
// Sizes: 96 MiB (inside the 256 MiB Infinity Cache after the first touch, like C2's working set)
// and 768 MiB (past it).  Every kernel runs 3 times; the per-dispatch counters are compared with
// the byte count by tools/micro/fetch_calib_summary.py.
//   hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d out -o run -- ./fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

template <class T>
__global__ void __launch_bounds__(256) k_read(const T *__restrict__ a, int64_t n, double *__restrict__ sink) {
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        if constexpr (sizeof(T) == 16) acc += a[i].x + a[i].y;
        else acc += (double)a[i];
    }
    if (acc == 12345.678) sink[0] = acc;      // never true: keeps the loads
}

__global__ void __launch_bounds__(256) k_gather(const double *__restrict__ a, const int32_t *__restrict__ idx, int64_t n,
                                                double *__restrict__ sink) {
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) acc += a[idx[i]];
    if (acc == 12345.678) sink[0] = acc;
}

template <class T>
__global__ void __launch_bounds__(256) k_write(T *__restrict__ a, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        if constexpr (sizeof(T) == 16) a[i] = make_double2((double)i, 1.0);
        else a[i] = (T)i;
    }
}

int main() {
    const int64_t sizes[2] = {96ll << 20, 768ll << 20};
    double *sink;
    CK(hipMalloc(&sink, 8));
    const int grid = 256 * 8 * 4;
    for (int64_t bytes : sizes) {
        void *buf;
        int32_t *idx;
        CK(hipMalloc(&buf, bytes));
        CK(hipMemset(buf, 0, bytes));
        const int64_t n8 = bytes / 8;
        // phase-2-like gather: a block-local shuffle (neighbouring rows' edges): 4096-element windows
        std::vector<int32_t> h(n8 / 2);
        for (int64_t i = 0; i < (int64_t)h.size(); i++) {
            const int64_t w = i & ~4095ll, o = i & 4095;
            h[i] = (int32_t)(w + ((o * 2654435761ll) & 4095));
        }
        CK(hipMalloc(&idx, sizeof(int32_t) * h.size()));
        CK(hipMemcpy(idx, h.data(), sizeof(int32_t) * h.size(), hipMemcpyHostToDevice));
        for (int rep = 0; rep < 3; rep++) {
            k_read<float><<<grid, 256>>>((const float *)buf, bytes / 4, sink);
            k_read<double><<<grid, 256>>>((const double *)buf, bytes / 8, sink);
            k_read<double2><<<grid, 256>>>((const double2 *)buf, bytes / 16, sink);
            k_gather<<<grid, 256>>>((const double *)buf, idx, (int64_t)h.size(), sink);
            k_write<double><<<grid, 256>>>((double *)buf, bytes / 8);
            k_write<double2><<<grid, 256>>>((double2 *)buf, bytes / 16);
        }
        CK(hipDeviceSynchronize());
        std::printf("size %lld bytes: read4 read8 read16 gather8 (%lld gathered doubles + %lld index bytes) write8 write16, x3\n",
                    (long long)bytes, (long long)h.size(), (long long)(4 * h.size()));
        CK(hipFree(buf));
        CK(hipFree(idx));
    }
    return 0;
}
