// graph_dev.hip — computeR (Modules/Utils/Geometry.cc:549-604) on the device: one thread per mesh
// vertex of a keyframe pair, the cross-covariance over its CSR neighbours and Eigen's Jacobi SVD
// restated in procrustes.h (shared with the host loop in graph_builder.cpp).  Built with
// -ffp-contract=off and IEEE fp64 division/sqrt so the rotations equal the host's bit for bit
// (tests/test_graph_gpu.py).  The work is ~1 us of fp64 per vertex and independent per vertex:
// latency-bound on the host (100k vertices ~ 0.1 s on one core), a few tens of us here.
#include "graph_builder.h"
#include "procrustes.h"

namespace deftri {

namespace {
constexpr int kRBlock = 256;

__global__ __launch_bounds__(kRBlock) void k_compute_r(int n1, int n2, const int32_t *__restrict__ off,
                                                       const int32_t *__restrict__ adj, const double *__restrict__ w,
                                                       const int32_t *__restrict__ pos_idx,
                                                       const int32_t *__restrict__ inv, const double *__restrict__ pos1,
                                                       const double *__restrict__ pos2, double *__restrict__ R) {
    const int i = blockIdx.x * kRBlock + threadIdx.x;
    if (i >= n1) return;
    double r[9];
    compute_r_vertex(i, n2, off, adj, w, pos_idx, inv, pos1, pos2, r);
    for (int k = 0; k < 9; k++) R[9 * (size_t)i + k] = r[k];
}

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

GraphDevice::~GraphDevice() {
    if (buf_) {
        hipSetDevice(dev_);
        hipStreamSynchronize(st_);
        hipFree(buf_);
    }
}

bool GraphDevice::compute_r(int n1, int n2, const int32_t *off, const int32_t *adj, const double *w, int64_t nadj,
                            const int32_t *pos_idx, const int32_t *inv, const double *pos1, const double *pos2,
                            double *R, std::string &err) {
    if (n1 <= 0) return true;
    hipSetDevice(dev_);
    const size_t b_w = align_up(sizeof(double) * (size_t)std::max<int64_t>(nadj, 1));
    const size_t b_p1 = align_up(sizeof(double) * 3 * (size_t)n1), b_p2 = align_up(sizeof(double) * 3 * (size_t)std::max(n2, 1));
    const size_t b_r = align_up(sizeof(double) * 9 * (size_t)n1);
    const size_t b_off = align_up(sizeof(int32_t) * (size_t)(n1 + 1)), b_adj = align_up(sizeof(int32_t) * (size_t)std::max<int64_t>(nadj, 1));
    const size_t b_n = align_up(sizeof(int32_t) * (size_t)n1);
    const size_t need = b_w + b_p1 + b_p2 + b_r + b_off + b_adj + 2 * b_n;
    auto check = [&](hipError_t e, const char *what) {
        if (e != hipSuccess) err = std::string("computeR on the device: ") + what + ": " + hipGetErrorString(e);
        return e == hipSuccess;
    };
    if (need > cap_) {
        if (buf_) { hipStreamSynchronize(st_); hipFree(buf_); buf_ = nullptr; cap_ = 0; }
        if (!check(hipMalloc(&buf_, need), "hipMalloc")) return false;
        cap_ = need;
    }
    char *b = static_cast<char *>(buf_);
    double *dw = (double *)b; b += b_w;
    double *dp1 = (double *)b; b += b_p1;
    double *dp2 = (double *)b; b += b_p2;
    double *dR = (double *)b; b += b_r;
    int32_t *doff = (int32_t *)b; b += b_off;
    int32_t *dadj = (int32_t *)b; b += b_adj;
    int32_t *dpi = (int32_t *)b; b += b_n;
    int32_t *dinv = (int32_t *)b;
    const hipMemcpyKind h2d = hipMemcpyHostToDevice;
    if (!check(hipMemcpyAsync(dw, w, sizeof(double) * (size_t)nadj, h2d, st_), "copy") ||
        !check(hipMemcpyAsync(dp1, pos1, sizeof(double) * 3 * (size_t)n1, h2d, st_), "copy") ||
        !check(hipMemcpyAsync(dp2, pos2, sizeof(double) * 3 * (size_t)n2, h2d, st_), "copy") ||
        !check(hipMemcpyAsync(doff, off, sizeof(int32_t) * (size_t)(n1 + 1), h2d, st_), "copy") ||
        !check(hipMemcpyAsync(dadj, adj, sizeof(int32_t) * (size_t)nadj, h2d, st_), "copy") ||
        !check(hipMemcpyAsync(dpi, pos_idx, sizeof(int32_t) * (size_t)n1, h2d, st_), "copy") ||
        !check(hipMemcpyAsync(dinv, inv, sizeof(int32_t) * (size_t)n1, h2d, st_), "copy"))
        return false;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, st_);
    k_compute_r<<<(n1 + kRBlock - 1) / kRBlock, kRBlock, 0, st_>>>(n1, n2, doff, dadj, dw, dpi, dinv, dp1, dp2, dR);
    hipEventRecord(e1, st_);
    bool ok = check(hipGetLastError(), "launch") &&
              check(hipMemcpyAsync(R, dR, sizeof(double) * 9 * (size_t)n1, hipMemcpyDeviceToHost, st_), "copy back") &&
              check(hipStreamSynchronize(st_), "synchronize");
    float ms = 0;
    if (ok) hipEventElapsedTime(&ms, e0, e1);
    ms_last = ms;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ok;
}

}  // namespace deftri
