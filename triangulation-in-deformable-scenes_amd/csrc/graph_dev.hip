// graph_dev.hip — the per-pair geometry of the graph build on the device: the cotangent weights of
// the Delaunay mesh (ComputeEdgeWeightsCot, Modules/Utils/Geometry.cc:272-298) and computeR
// (Geometry.cc:549-604: per vertex the cross-covariance over its CSR neighbours and Eigen's Jacobi
// SVD), both restated in procrustes.h and shared with the host loops in graph_builder.cpp.  Built
// with -ffp-contract=off and IEEE fp64 division / sqrt so the weights and rotations equal the host's
// bit for bit (tests/test_graph_gpu.py).  computeR is ~1 us of fp64 per vertex: 48 ms for 100k
// vertices on one host core, ~50 us here.
#include "graph_builder.h"
#include "procrustes.h"

namespace deftri {

namespace {
constexpr int kRBlock = 256;

__device__ __forceinline__ int64_t csr_find(const int32_t *__restrict__ off, const int32_t *__restrict__ adj, int i, int j) {
    int lo = off[i], hi = off[i + 1];               // lower_bound in row i
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (adj[mid] < j) lo = mid + 1;
        else hi = mid;
    }
    return (lo < off[i + 1] && adj[lo] == j) ? lo : -1;
}

// one thread per triangle corner: the cot term of the edge opposite the corner into one of the
// edge's two slots (an integer ticket picks the slot; a planar triangulation has at most two
// opposite corners per edge; more — duplicate or degenerate points — flags the pair, whose weights
// and rotations the host loops then compute: they average over every opposite corner, as
// Geometry.cc:283-290 does)
__global__ __launch_bounds__(kRBlock) void k_cot_corners(int ntri, const int32_t *__restrict__ tris,
                                                         const int32_t *__restrict__ off, const int32_t *__restrict__ adj,
                                                         const double *__restrict__ pos, double *__restrict__ slot,
                                                         int *__restrict__ cnt, int *__restrict__ bad) {
    const int64_t t3 = (int64_t)blockIdx.x * kRBlock + threadIdx.x;
    if (t3 >= 3 * (int64_t)ntri) return;
    const int64_t t = t3 / 3;
    const int k = (int)(t3 - 3 * t);
    const int v0 = tris[3 * t + k], v1 = tris[3 * t + (k + 1) % 3], v2 = tris[3 * t + (k + 2) % 3];
    const int e0 = min(v0, v1), e1 = max(v0, v1);
    const int64_t at = csr_find(off, adj, e0, e1);
    if (at < 0) { atomicExch(bad, 1); return; }
    const double c = cot_term(pos + 3 * (int64_t)e0, pos + 3 * (int64_t)e1, pos + 3 * (int64_t)v2);
    const int sidx = atomicAdd(cnt + at, 1);
    if (sidx > 1) { atomicExch(bad, 1); return; }
    slot[2 * at + sidx] = c;
}

// one thread per vertex: its entries to higher-numbered neighbours get the mean of their slots
// ((0 + s0) + s1, the host loop's sum: two terms add the same either way), clamped, mirrored
__global__ __launch_bounds__(kRBlock) void k_cot_finish(int n, const int32_t *__restrict__ off, const int32_t *__restrict__ adj,
                                                        const double *__restrict__ slot, const int *__restrict__ cnt,
                                                        double *__restrict__ w) {
    const int i = blockIdx.x * kRBlock + threadIdx.x;
    if (i >= n) return;
    for (int32_t k = off[i]; k < off[i + 1]; k++) {
        const int j = adj[k];
        if (j < i) continue;
        const int c = cnt[k];
        double sum = 0.0;
        if (c > 0) sum += slot[2 * (int64_t)k];
        if (c > 1) sum += slot[2 * (int64_t)k + 1];
        const double wt = cot_weight(sum, c);
        w[k] = wt;
        w[csr_find(off, adj, j, i)] = wt;
    }
}

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

int GraphDevice::mesh_pass(int n1, int n2, const int32_t *tris, int ntri, const int32_t *off, const int32_t *adj,
                           int64_t nadj, const int32_t *pos_idx, const int32_t *inv, const double *pos1,
                           const double *pos2, double *w_out, double *R, std::string &err) {
    if (n1 <= 0) return 0;
    hipSetDevice(dev_);
    const size_t na = (size_t)std::max<int64_t>(nadj, 1);
    const size_t b_w = align_up(sizeof(double) * na), b_slot = align_up(2 * sizeof(double) * na);
    const size_t b_p1 = align_up(sizeof(double) * 3 * (size_t)n1), b_p2 = align_up(sizeof(double) * 3 * (size_t)std::max(n2, 1));
    const size_t b_r = align_up(sizeof(double) * 9 * (size_t)n1);
    const size_t b_tri = align_up(sizeof(int32_t) * 3 * (size_t)std::max(ntri, 1));
    const size_t b_off = align_up(sizeof(int32_t) * (size_t)(n1 + 1)), b_adj = align_up(sizeof(int32_t) * na);
    const size_t b_cnt = align_up(sizeof(int) * (na + 1));
    const size_t b_n = align_up(sizeof(int32_t) * (size_t)n1);
    const size_t need = b_w + b_slot + b_p1 + b_p2 + b_r + b_tri + b_off + b_adj + b_cnt + 2 * b_n;
    auto check = [&](hipError_t e, const char *what) {
        if (e != hipSuccess) err = std::string("graph geometry on the device: ") + what + ": " + hipGetErrorString(e);
        return e == hipSuccess;
    };
    if (need > cap_) {
        if (buf_) { hipStreamSynchronize(st_); hipFree(buf_); buf_ = nullptr; cap_ = 0; }
        if (!check(hipMalloc(&buf_, need), "hipMalloc")) return -1;
        cap_ = need;
    }
    char *b = static_cast<char *>(buf_);
    double *dw = (double *)b; b += b_w;
    double *dslot = (double *)b; b += b_slot;
    double *dp1 = (double *)b; b += b_p1;
    double *dp2 = (double *)b; b += b_p2;
    double *dR = (double *)b; b += b_r;
    int32_t *dtri = (int32_t *)b; b += b_tri;
    int32_t *doff = (int32_t *)b; b += b_off;
    int32_t *dadj = (int32_t *)b; b += b_adj;
    int *dcnt = (int *)b; b += b_cnt;            // [nadj] slot tickets, [nadj] the error flag
    int32_t *dpi = (int32_t *)b; b += b_n;
    int32_t *dinv = (int32_t *)b;
    const hipMemcpyKind h2d = hipMemcpyHostToDevice;
    if (!check(hipMemcpyAsync(dp1, pos1, sizeof(double) * 3 * (size_t)n1, h2d, st_), "copy") ||
        !check(hipMemcpyAsync(dp2, pos2, sizeof(double) * 3 * (size_t)n2, h2d, st_), "copy") ||
        !check(hipMemcpyAsync(dtri, tris, sizeof(int32_t) * 3 * (size_t)ntri, h2d, st_), "copy") ||
        !check(hipMemcpyAsync(doff, off, sizeof(int32_t) * (size_t)(n1 + 1), h2d, st_), "copy") ||
        !check(hipMemcpyAsync(dadj, adj, sizeof(int32_t) * (size_t)nadj, h2d, st_), "copy") ||
        !check(hipMemcpyAsync(dpi, pos_idx, sizeof(int32_t) * (size_t)n1, h2d, st_), "copy") ||
        !check(hipMemcpyAsync(dinv, inv, sizeof(int32_t) * (size_t)n1, h2d, st_), "copy") ||
        !check(hipMemsetAsync(dcnt, 0, sizeof(int) * (na + 1), st_), "memset"))
        return -1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, st_);
    const int64_t corners = 3 * (int64_t)ntri;
    if (corners > 0)
        k_cot_corners<<<(unsigned)((corners + kRBlock - 1) / kRBlock), kRBlock, 0, st_>>>(ntri, dtri, doff, dadj, dp1, dslot,
                                                                                           dcnt, dcnt + na);
    k_cot_finish<<<(n1 + kRBlock - 1) / kRBlock, kRBlock, 0, st_>>>(n1, doff, dadj, dslot, dcnt, dw);
    k_compute_r<<<(n1 + kRBlock - 1) / kRBlock, kRBlock, 0, st_>>>(n1, n2, doff, dadj, dw, dpi, dinv, dp1, dp2, dR);
    hipEventRecord(e1, st_);
    int bad = 0;
    bool ok = check(hipGetLastError(), "launch") &&
              check(hipMemcpyAsync(w_out, dw, sizeof(double) * (size_t)nadj, hipMemcpyDeviceToHost, st_), "copy back") &&
              check(hipMemcpyAsync(R, dR, sizeof(double) * 9 * (size_t)n1, hipMemcpyDeviceToHost, st_), "copy back") &&
              check(hipMemcpyAsync(&bad, dcnt + na, sizeof(int), hipMemcpyDeviceToHost, st_), "copy back") &&
              check(hipStreamSynchronize(st_), "synchronize");
    float ms = 0;
    if (ok) hipEventElapsedTime(&ms, e0, e1);
    ms_last = ms;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    if (!ok) return -1;
    return bad ? 1 : 0;      // 1: an edge with more than two opposite vertices — the host loops redo the pair
}

}  // namespace deftri
