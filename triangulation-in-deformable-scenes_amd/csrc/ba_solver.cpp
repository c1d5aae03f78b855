// ba_solver.cpp — C-ABI of the bundle-adjustment LM path (include/deftri.h, "bundle adjustment").
//
// Restates, on the device, what the reference's BA entry points hand to g2o
// (Modules/Optimization/g2oBundleAdjustment.cc:38-444):
//   optimizer.initializeOptimization(level)   active edges = level `level` with a non-fixed
//                                             vertex; active vertices = vertices of active edges
//   optimizer.optimize(n)                     OptimizationAlgorithmLevenberg over BlockSolver_6_3:
//                                             points marginalized (Schur), LinearSolverEigen on Hschur
// with the g2o LM control flow of solver.cpp (tau 1e-5, rho rule, nu doubling, <= 10 trials).
// Edges are stored in point order on the device (CSR); every per-edge array of the C-ABI uses the
// caller's edge order (perm).
//
// Multi-GPU (point sharding): each rank holds every pose and a disjoint subset of the points with
// their edges.  Per LM iteration the pose blocks {chi2, Hpp, bp} are summed over ranks; per trial
// the Schur partial {-sum Hpl Dinv Hlp, -sum Hpl Dinv bl} and the scalars {chi2_new, scale} are
// summed (RCCL all-reduce on the solver stream).  The reduced pose system is then solved
// identically on every rank, and each rank back-substitutes its own points.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/deftri.h"
#include "ba.h"
#include "exit_guard.h"

using namespace deftri;

struct deftri_ba_ctx {
    int device = 0;
    hipStream_t st = nullptr;
    hipEvent_t ev[8]{};
    std::string err;
    bool have = false;
    BADev B;
    std::vector<void *> allocs;
    // host copies (caller order unless noted)
    int32_t K = 0, P = 0, E = 0;
    std::vector<double> poses0, points0;
    std::vector<uint8_t> pose_fixed, point_fixed;
    std::vector<uint8_t> level, robust;       // caller order
    std::vector<int32_t> perm;                // sorted edge -> caller edge
    std::vector<int32_t> e_point, e_pose;     // sorted order
    std::vector<int32_t> lead;                // sorted order
    int32_t *d_perm = nullptr;
    // Schur buffers are sized for the largest ns seen so far
    int32_t cap_ns = -1;
    double *hb = nullptr;                     // [1 + 42K]: chi2, Hpp, bp (one all-reduce)
    // distribution
    int32_t nranks = 1, rank = 0;
    ncclComm_t comm = nullptr;
    deftri_allreduce_fn fn = nullptr;
    void *fn_user = nullptr;
    std::vector<double> stage;                // host staging for the callback all-reduce
    double *hpin = nullptr;                   // pinned host staging of the per-trial scalars
    int *ipin = nullptr;
    int32_t n_free_points = 0;
    int64_t n_free_points_global = 0;        // summed over the point shards
};

namespace {

int fail(deftri_ba_ctx *c, int code, const std::string &m) {
    if (c) c->err = m;
    return code;
}

#define HIPOK(expr)                                                                          \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail(ctx, DEFTRI_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class T>
int dalloc(deftri_ba_ctx *ctx, T **p, int64_t n) {
    *p = nullptr;
    if (n <= 0) n = 1;
    void *v = nullptr;
    hipError_t e = hipMalloc(&v, sizeof(T) * (size_t)n);
    if (e != hipSuccess) return fail(ctx, DEFTRI_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    ctx->allocs.push_back(v);
    *p = (T *)v;
    return 0;
}

template <class T>
int dput(deftri_ba_ctx *ctx, T **p, const T *h, int64_t n) {
    int rc = dalloc(ctx, p, n);
    if (rc) return rc;
    if (n > 0 && h) HIPOK(hipMemcpy(*p, h, sizeof(T) * (size_t)n, hipMemcpyHostToDevice));
    return 0;
}

template <class T>
int dput(deftri_ba_ctx *ctx, T **p, const std::vector<T> &v) { return dput(ctx, p, v.data(), (int64_t)v.size()); }

void free_device(deftri_ba_ctx *ctx) {
    for (void *p : ctx->allocs) hipFree(p);
    ctx->allocs.clear();
    ctx->B = BADev();
    ctx->hb = nullptr;
    ctx->d_perm = nullptr;
    ctx->cap_ns = -1;
    ctx->have = false;
}

// in-place sum / max over ranks of n device doubles (no-op on one rank)
int allreduce(deftri_ba_ctx *ctx, double *buf, int64_t n, int op) {
    if (n <= 0) return 0;
    if (ctx->comm) {                          // RCCL (also with one rank: exercises the path)
        ncclResult_t r = ncclAllReduce(buf, buf, (size_t)n, ncclDouble, op == 0 ? ncclSum : ncclMax, ctx->comm, ctx->st);
        if (r != ncclSuccess) return fail(ctx, DEFTRI_E_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
        return 0;
    }
    if (ctx->nranks <= 1) return 0;
    if (!ctx->fn) return fail(ctx, DEFTRI_E_ARG, "distributed context without a transport");
    if ((int64_t)ctx->stage.size() < n) ctx->stage.resize((size_t)n);
    HIPOK(hipMemcpyAsync(ctx->stage.data(), buf, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, ctx->st));
    HIPOK(hipStreamSynchronize(ctx->st));
    if (ctx->fn(ctx->fn_user, ctx->stage.data(), n, op) != 0) return fail(ctx, DEFTRI_E_ARG, "all-reduce callback failed");
    HIPOK(hipMemcpyAsync(buf, ctx->stage.data(), sizeof(double) * (size_t)n, hipMemcpyHostToDevice, ctx->st));
    return 0;
}

int validate(deftri_ba_ctx *ctx, const deftri_ba_desc *d) {
    if (!d) return fail(ctx, DEFTRI_E_ARG, "null descriptor");
    if (d->n_poses < 0 || d->n_points < 0 || d->n_edges < 0) return fail(ctx, DEFTRI_E_ARG, "negative count");
    if ((d->n_poses && (!d->poses || !d->pose_kb8)) || (d->n_points && !d->points) ||
        (d->n_edges && (!d->edge_point || !d->edge_pose || !d->edge_obs || !d->edge_info)))
        return fail(ctx, DEFTRI_E_ARG, "missing array");
    for (int32_t e = 0; e < d->n_edges; e++) {
        if (d->edge_point[e] < 0 || d->edge_point[e] >= d->n_points)
            return fail(ctx, DEFTRI_E_ARG, "edge_point out of range at edge " + std::to_string(e));
        if (d->edge_pose[e] < 0 || d->edge_pose[e] >= d->n_poses)
            return fail(ctx, DEFTRI_E_ARG, "edge_pose out of range at edge " + std::to_string(e));
    }
    return 0;
}

// initializeOptimization(level): activity of edges and vertices, Schur indices, LDS tables.
int prepare_active(deftri_ba_ctx *ctx, int32_t level) {
    // initializeOptimization(level) on the device: the edge / vertex activity is computed by
    // kernels; only the K pose flags come to the host (Schur slots of the free poses, K <= 200)
    BADev &B = ctx->B;
    const int32_t K = ctx->K, P = ctx->P;
    if (level < 0 || level > 255) return fail(ctx, DEFTRI_E_ARG, "level out of range");
    ba_launch_active(B, level, ctx->st);
    std::vector<int32_t> pflag(std::max(K, 1), 0);
    if (K > 0) HIPOK(hipMemcpyAsync(pflag.data(), B.pose_flag, sizeof(int32_t) * K, hipMemcpyDeviceToHost, ctx->st));
    HIPOK(hipStreamSynchronize(ctx->st));
    std::vector<double> pose_cnt(K, 0.0);
    for (int32_t k = 0; k < K; k++) pose_cnt[k] = pflag[k] ? 1.0 : 0.0;
    if ((ctx->nranks > 1 || ctx->comm) && K > 0) {   // a pose is active if any rank holds an active edge of it
        double *d = B.Spart;                 // scratch (allocated with >= K doubles at upload)
        HIPOK(hipMemcpyAsync(d, pose_cnt.data(), sizeof(double) * K, hipMemcpyHostToDevice, ctx->st));
        int rc = allreduce(ctx, d, K, 0);
        if (rc) return rc;
        HIPOK(hipMemcpyAsync(pose_cnt.data(), d, sizeof(double) * K, hipMemcpyDeviceToHost, ctx->st));
        HIPOK(hipStreamSynchronize(ctx->st));
    }
    std::vector<int32_t> sidx(std::max(K, 1), -1);
    int32_t nfree = 0;
    for (int32_t k = 0; k < K; k++)
        if (pose_cnt[k] > 0 && !ctx->pose_fixed[k]) sidx[k] = nfree++;
    if (nfree > 200) return fail(ctx, DEFTRI_E_ARG, "more than 200 free poses in one Schur system");
    if (K > 0) HIPOK(hipMemcpyAsync(B.pose_sidx, sidx.data(), sizeof(int32_t) * K, hipMemcpyHostToDevice, ctx->st));
    ba_launch_free_slots(B, ctx->st);
    int32_t *nfp_h = ctx->ipin + 1;          // pinned
    HIPOK(hipMemcpyAsync(nfp_h, B.icount, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->st));
    HIPOK(hipMemsetAsync(B.dxl, 0, sizeof(double) * 3 * (size_t)std::max(P, 1), ctx->st));
    HIPOK(hipStreamSynchronize(ctx->st));
    const int32_t nfp = *nfp_h;
    // the pose-solve rule and the nothing-to-optimize exit must agree on every rank: they follow the
    // free points of the whole graph, not of this rank's shard
    int64_t nfp_global = nfp;
    if (ctx->nranks > 1 || ctx->comm) {
        double *d = B.Spart;
        ctx->hpin[8] = (double)nfp;
        HIPOK(hipMemcpyAsync(d, ctx->hpin + 8, sizeof(double), hipMemcpyHostToDevice, ctx->st));
        int rc = allreduce(ctx, d, 1, 0);
        if (rc) return rc;
        HIPOK(hipMemcpyAsync(ctx->hpin + 8, d, sizeof(double), hipMemcpyDeviceToHost, ctx->st));
        HIPOK(hipStreamSynchronize(ctx->st));
        nfp_global = (int64_t)ctx->hpin[8];
    }
    B.nfree = nfree;
    B.ns = 6 * nfree;
    B.dense_positive = nfp_global == 0 ? 1 : 0;   // poses only: LinearSolverDense (Eigen LDLT, isPositive)
    ctx->n_free_points = nfp;
    ctx->n_free_points_global = nfp_global;
    const int64_t NE = (int64_t)B.ns * (B.ns + 1) / 2 + B.ns;
    if (B.ns > ctx->cap_ns) {
        int rc;
        const int64_t grp = std::max<int64_t>(std::max(B.ngroup, B.mgroup), 1);
        if ((rc = dalloc(ctx, &B.Spart, std::max<int64_t>(grp * NE, K)))) return rc;
        if ((rc = dalloc(ctx, &B.Sred, NE))) return rc;
        if ((rc = dalloc(ctx, &B.S, (int64_t)B.ns * B.ns))) return rc;
        if ((rc = dalloc(ctx, &B.xp, std::max(B.ns, 1)))) return rc;
        ctx->cap_ns = B.ns;
    }
    return 0;
}

// edge levels (original edge order) -> device, point order
int upload_levels(deftri_ba_ctx *ctx) {
    std::vector<uint8_t> lv(std::max(ctx->E, 1));
    for (int32_t s = 0; s < ctx->E; s++) lv[s] = ctx->level[ctx->perm[s]];
    HIPOK(hipMemcpyAsync(ctx->B.e_level, lv.data(), ctx->E, hipMemcpyHostToDevice, ctx->st));
    HIPOK(hipStreamSynchronize(ctx->st));
    return 0;
}

// computeActiveErrors + activeRobustChi2 (this rank) -> dst; with Jacobians: buildSystem
void linearize(deftri_ba_ctx *ctx, bool want_jac, double *chi_dst) {
    BADev &B = ctx->B;
    ba_launch_edges(B, ctx->st, want_jac, false);
    ba_launch_chi2_sum(B, chi_dst, ctx->st);
    if (want_jac) {
        ba_launch_points(B, ctx->st);
        ba_launch_poses(B, ctx->st);
    }
}

void push_state(deftri_ba_ctx *ctx) {
    BADev &B = ctx->B;
    hipMemcpyAsync(B.points_bak, B.points, sizeof(double) * 3 * (size_t)B.P, hipMemcpyDeviceToDevice, ctx->st);
    hipMemcpyAsync(B.poses_bak, B.poses, sizeof(double) * 7 * (size_t)B.K, hipMemcpyDeviceToDevice, ctx->st);
}

void pop_state(deftri_ba_ctx *ctx) {
    BADev &B = ctx->B;
    hipMemcpyAsync(B.points, B.points_bak, sizeof(double) * 3 * (size_t)B.P, hipMemcpyDeviceToDevice, ctx->st);
    hipMemcpyAsync(B.poses, B.poses_bak, sizeof(double) * 7 * (size_t)B.K, hipMemcpyDeviceToDevice, ctx->st);
}

float ev_ms(deftri_ba_ctx *ctx, int a, int b) {
    float ms = 0;
    hipEventElapsedTime(&ms, ctx->ev[a], ctx->ev[b]);
    return ms;
}

}  // namespace

using LiveBa = deftri::LiveContexts<deftri_ba_ctx, deftri_ba_destroy>;

extern "C" {

int deftri_ba_create(int32_t device, deftri_ba_ctx **out) {
    if (!out) return DEFTRI_E_ARG;
    *out = nullptr;
    int n = 0;
    if (device < 0 || hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device >= n) return DEFTRI_E_NODEVICE;
    deftri_ba_ctx *ctx = new deftri_ba_ctx();
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->st, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return DEFTRI_E_HIP;
    }
    for (auto &e : ctx->ev) hipEventCreate(&e);
    if (hipHostMalloc((void **)&ctx->hpin, 16 * sizeof(double), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&ctx->ipin, 16 * sizeof(int), hipHostMallocDefault) != hipSuccess) {
        delete ctx;
        return DEFTRI_E_HIP;
    }
    LiveBa::add(ctx);
    *out = ctx;
    return 0;
}

int deftri_ba_destroy(deftri_ba_ctx *ctx) {
    if (!ctx) return 0;
    LiveBa::remove(ctx);
    hipSetDevice(ctx->device);
    if (ctx->st) hipStreamSynchronize(ctx->st);
    free_device(ctx);
    if (ctx->comm) ncclCommDestroy(ctx->comm);
    for (auto &e : ctx->ev) if (e) hipEventDestroy(e);
    if (ctx->st) hipStreamDestroy(ctx->st);
    if (ctx->hpin) hipHostFree(ctx->hpin);
    if (ctx->ipin) hipHostFree(ctx->ipin);
    delete ctx;
    return 0;
}

const char *deftri_ba_last_error(const deftri_ba_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int deftri_ba_upload(deftri_ba_ctx *ctx, const deftri_ba_desc *d) {
    if (!ctx) return DEFTRI_E_ARG;
    int rc = validate(ctx, d);
    if (rc) return rc;
    hipSetDevice(ctx->device);
    HIPOK(hipStreamSynchronize(ctx->st));
    free_device(ctx);
    const int32_t K = d->n_poses, P = d->n_points, E = d->n_edges;
    ctx->K = K; ctx->P = P; ctx->E = E;
    ctx->poses0.assign(d->poses, d->poses + 7 * (size_t)K);
    ctx->points0.assign(d->points, d->points + 3 * (size_t)P);
    ctx->pose_fixed.assign(K, 0);
    if (d->pose_fixed) ctx->pose_fixed.assign(d->pose_fixed, d->pose_fixed + K);
    ctx->point_fixed.assign(P, 0);
    if (d->point_fixed) ctx->point_fixed.assign(d->point_fixed, d->point_fixed + P);
    ctx->level.assign(E, 0);
    if (d->edge_level) ctx->level.assign(d->edge_level, d->edge_level + E);
    ctx->robust.assign(E, 1);
    if (d->edge_robust) ctx->robust.assign(d->edge_robust, d->edge_robust + E);
    // edges in point order (stable), CSR point -> edges
    ctx->perm.resize(E);
    std::iota(ctx->perm.begin(), ctx->perm.end(), 0);
    std::stable_sort(ctx->perm.begin(), ctx->perm.end(),
                     [&](int32_t a, int32_t b) { return d->edge_point[a] < d->edge_point[b]; });
    std::vector<int32_t> pt_ptr(P + 1, 0);
    ctx->e_point.resize(E); ctx->e_pose.resize(E);
    std::vector<double> obs(2 * (size_t)E), info(E);
    std::vector<uint8_t> rob(E);
    for (int32_t s = 0; s < E; s++) {
        const int32_t o = ctx->perm[s];
        ctx->e_point[s] = d->edge_point[o];
        ctx->e_pose[s] = d->edge_pose[o];
        obs[2 * (size_t)s] = d->edge_obs[2 * (size_t)o];
        obs[2 * (size_t)s + 1] = d->edge_obs[2 * (size_t)o + 1];
        info[s] = d->edge_info[o];
        rob[s] = ctx->robust[o];
        pt_ptr[ctx->e_point[s] + 1]++;
    }
    for (int32_t l = 0; l < P; l++) pt_ptr[l + 1] += pt_ptr[l];
    // lead edge of each (point, pose) pair
    ctx->lead.resize(E);
    for (int32_t l = 0; l < P; l++) {
        if (pt_ptr[l + 1] - pt_ptr[l] > kBaStageEdges)
            return fail(ctx, DEFTRI_E_ARG, "a point has more than " + std::to_string(kBaStageEdges) + " observations");
        for (int32_t s = pt_ptr[l]; s < pt_ptr[l + 1]; s++) {
            ctx->lead[s] = s;
            for (int32_t q = pt_ptr[l]; q < s; q++)
                if (ctx->e_pose[q] == ctx->e_pose[s]) { ctx->lead[s] = ctx->lead[q]; break; }
        }
    }
    // pose -> edges (sorted edge ids) and 256-edge chunks
    std::vector<int32_t> pose_ptr(K + 1, 0), pose_edges(E);
    for (int32_t s = 0; s < E; s++) pose_ptr[ctx->e_pose[s] + 1]++;
    for (int32_t k = 0; k < K; k++) pose_ptr[k + 1] += pose_ptr[k];
    {
        std::vector<int32_t> fill(pose_ptr.begin(), pose_ptr.end() - 1);
        for (int32_t s = 0; s < E; s++) pose_edges[fill[ctx->e_pose[s]]++] = s;
    }
    std::vector<int32_t> chunk_beg, chunk_len, pose_chunk_ptr(K + 1, 0);
    for (int32_t k = 0; k < K; k++) {
        for (int32_t b = pose_ptr[k]; b < pose_ptr[k + 1]; b += kBaPoseChunk) {
            chunk_beg.push_back(b);
            chunk_len.push_back(std::min(kBaPoseChunk, pose_ptr[k + 1] - b));
        }
        pose_chunk_ptr[k + 1] = (int32_t)chunk_beg.size();
    }
    // Schur-GEMM stages (point ranges with <= kBaStageEdges edges) and workgroup groups
    std::vector<int32_t> stage_pt{0};
    for (int32_t l = 0; l < P; l++) {
        const int32_t ne = pt_ptr[l + 1] - pt_ptr[stage_pt.back()];
        if (ne > kBaStageEdges) stage_pt.push_back(l);
    }
    if (stage_pt.back() != P) stage_pt.push_back(P);
    const int32_t nstage = (int32_t)stage_pt.size() - 1;
    // at most 512 workgroup groups, and at most 16M doubles of per-group partial systems
    const int64_t ns_max = 6 * (int64_t)K, ne_max = ns_max * (ns_max + 1) / 2 + ns_max;
    const int64_t max_groups = std::max<int64_t>(1, std::min<int64_t>(512, (16ll << 20) / std::max<int64_t>(ne_max, 1)));
    const int32_t per_group = (int32_t)std::max<int64_t>(1, (nstage + max_groups - 1) / max_groups);
    std::vector<int32_t> group_stage;
    for (int32_t s = 0; s < nstage; s += per_group) group_stage.push_back(s);
    group_stage.push_back(nstage);
    // MFMA path: 16-point stages grouped per workgroup (about 1024 groups)
    const int32_t nmstage = (P + 15) / 16;
    const int64_t max_mgroups = std::max<int64_t>(1, std::min<int64_t>(1024, (16ll << 20) / std::max<int64_t>(ne_max, 1)));
    const int32_t mper = (int32_t)std::max<int64_t>(1, (nmstage + max_mgroups - 1) / max_mgroups);
    BADev &B = ctx->B;
    B.mstages_per_group = mper;
    B.mgroup = P > 0 ? (nmstage + mper - 1) / mper : 0;
    B.K = K; B.P = P; B.E = E;
    B.huber = d->huber_delta;
    B.nchunk = (int32_t)chunk_beg.size();
    B.nstage = nstage;
    B.ngroup = P > 0 ? (int32_t)group_stage.size() - 1 : 0;
    std::vector<float> kb8(d->pose_kb8, d->pose_kb8 + 8 * (size_t)K);
#define PUT(dst, src) if ((rc = dput(ctx, &(dst), src))) return rc
#define ALLOC(dst, n) if ((rc = dalloc(ctx, &(dst), n))) return rc
    PUT(B.poses, ctx->poses0); ALLOC(B.poses_bak, 7 * (int64_t)K);
    PUT(B.points, ctx->points0); ALLOC(B.points_bak, 3 * (int64_t)P);
    PUT(B.kb8, kb8);
    PUT(B.e_point, ctx->e_point); PUT(B.e_pose, ctx->e_pose);
    PUT(B.obs, obs); PUT(B.info, info); PUT(B.robust, rob);
    ALLOC(B.active, E);
    PUT(B.pt_ptr, pt_ptr);
    ALLOC(B.pt_free, P);
    ALLOC(B.pose_sidx, K);
    PUT(B.pose_edges, pose_edges);
    PUT(B.chunk_beg, chunk_beg); PUT(B.chunk_len, chunk_len); PUT(B.pose_chunk_ptr, pose_chunk_ptr);
    PUT(B.stage_pt, stage_pt); PUT(B.group_stage, group_stage);
    ALLOC(B.pslot, E);
    PUT(B.lead, ctx->lead);
    ALLOC(B.e_level, E); ALLOC(B.pose_flag, K); ALLOC(B.pt_act, P); ALLOC(B.icount, 1);
    PUT(B.pt_fixed, ctx->point_fixed); PUT(B.pose_fixed, ctx->pose_fixed);
    ALLOC(B.err, 2 * (int64_t)E); ALLOC(B.wr, 2 * (int64_t)E);
    ALLOC(B.wgt, E); ALLOC(B.chi, E); ALLOC(B.chi2raw, E);
    ALLOC(B.Jp, 6 * (int64_t)E); ALLOC(B.JT, 12 * (int64_t)E);
    ALLOC(B.Wb, 18 * (int64_t)E); ALLOC(B.Y, 18 * (int64_t)E); ALLOC(B.v, 6 * (int64_t)E);
    ALLOC(B.Hll, 9 * (int64_t)P); ALLOC(B.bl, 3 * (int64_t)P); ALLOC(B.dbl, 3 * (int64_t)P); ALLOC(B.Dinv, 9 * (int64_t)P); ALLOC(B.dxl, 3 * (int64_t)P);
    ALLOC(B.pchunk, 27 * (int64_t)std::max(B.nchunk, 1));
    ALLOC(ctx->hb, 1 + 42 * (int64_t)K);
    B.Hpp = ctx->hb + 1;
    B.bp = ctx->hb + 1 + 36 * (int64_t)K;
    ALLOC(B.dxp, 6 * (int64_t)K);
    ALLOC(B.flag, 1);
    ALLOC(B.part, 512);
    ALLOC(B.scal, 8);
    {
        std::vector<int32_t> perm(ctx->perm);
        PUT(ctx->d_perm, perm);
    }
    // Schur scratch for the all-pose-free system (re-sized in prepare_active if needed)
    const int64_t ns = 6 * (int64_t)K, NE = ns * (ns + 1) / 2 + ns;
    ALLOC(B.Spart, std::max<int64_t>((int64_t)std::max(std::max(B.ngroup, B.mgroup), 1) * NE, K));
    ALLOC(B.Sred, NE); ALLOC(B.S, ns * ns); ALLOC(B.xp, std::max<int64_t>(ns, 1));
    ctx->cap_ns = (int32_t)ns;
    if ((rc = upload_levels(ctx))) return rc;
#undef PUT
#undef ALLOC
    HIPOK(hipMemset(B.err, 0, sizeof(double) * 2 * (size_t)std::max(E, 1)));
    HIPOK(hipMemset(B.bl, 0, sizeof(double) * 3 * (size_t)std::max(P, 1)));
    HIPOK(hipMemset(B.Hll, 0, sizeof(double) * 9 * (size_t)std::max(P, 1)));
    HIPOK(hipMemset(B.Dinv, 0, sizeof(double) * 9 * (size_t)std::max(P, 1)));
    HIPOK(hipMemset(B.dxl, 0, sizeof(double) * 3 * (size_t)std::max(P, 1)));
    HIPOK(hipMemset(B.chi2raw, 0, sizeof(double) * (size_t)std::max(E, 1)));
    HIPOK(hipDeviceSynchronize());
    ctx->have = true;
    return 0;
}

int deftri_ba_set_state(deftri_ba_ctx *ctx, const double *poses, const double *points) {
    if (!ctx || !ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(ctx->device);
    if (poses) HIPOK(hipMemcpyAsync(ctx->B.poses, poses, sizeof(double) * 7 * (size_t)ctx->K, hipMemcpyHostToDevice, ctx->st));
    if (points) HIPOK(hipMemcpyAsync(ctx->B.points, points, sizeof(double) * 3 * (size_t)ctx->P, hipMemcpyHostToDevice, ctx->st));
    HIPOK(hipStreamSynchronize(ctx->st));
    return 0;
}

int deftri_ba_set_edge_flags(deftri_ba_ctx *ctx, const uint8_t *level, const uint8_t *robust) {
    if (!ctx || !ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(ctx->device);
    if (level) {
        ctx->level.assign(level, level + ctx->E);
        int rc = upload_levels(ctx);
        if (rc) return rc;
    }
    if (robust) {
        ctx->robust.assign(robust, robust + ctx->E);
        std::vector<uint8_t> rob(ctx->E);
        for (int32_t s = 0; s < ctx->E; s++) rob[s] = ctx->robust[ctx->perm[s]];
        HIPOK(hipMemcpyAsync(ctx->B.robust, rob.data(), ctx->E, hipMemcpyHostToDevice, ctx->st));
        HIPOK(hipStreamSynchronize(ctx->st));
    }
    return 0;
}

int deftri_ba_solve_lm(deftri_ba_ctx *ctx, const deftri_lm_params *prm, int32_t level, deftri_report *rep) {
    if (!ctx || !prm) return DEFTRI_E_ARG;
    if (!ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(ctx->device);
    deftri_report local{};
    deftri_report &R = rep ? *rep : local;
    std::memset(&R, 0, sizeof(R));
    int rc = prepare_active(ctx, level);
    if (rc) return rc;
    BADev &B = ctx->B;
    R.n_unknowns = B.ns + 3 * (int64_t)ctx->n_free_points;
    R.factor_flops = (double)B.ns * B.ns * B.ns / 3.0;
    R.n_fronts = 1;
    const int max_trials = prm->max_trials > 0 ? prm->max_trials : 10;
    const double tau = prm->tau > 0 ? prm->tau : 1e-5;
    auto t_start = std::chrono::steady_clock::now();
    if (B.ns == 0 && ctx->n_free_points_global == 0) {   // SparseOptimizer::optimize: nothing to optimize
        R.status = DEFTRI_STATUS_TERMINATE;
        return 0;
    }
    double lambda = 0, ni = 2;
    double t_lin = 0, t_fac = 0, t_sol = 0, t_upd = 0;
    int status = DEFTRI_STATUS_OK, it;
    double currentChi = 0;
    for (it = 0; it < prm->n_iterations; it++) {
        hipEventRecord(ctx->ev[0], ctx->st);
        linearize(ctx, true, ctx->hb);                            // computeActiveErrors, buildSystem
        if ((rc = allreduce(ctx, ctx->hb, 1 + 42 * (int64_t)B.K, 0))) return rc;
        if (it == 0) {
            ba_launch_maxdiag(B, B.scal + 2, ctx->st);
            if ((rc = allreduce(ctx, B.scal + 2, 1, 1))) return rc;
        }
        hipEventRecord(ctx->ev[1], ctx->st);
        double *head = ctx->hpin;            // pinned: a pageable readback costs ~100 us per call
        HIPOK(hipMemcpyAsync(&head[0], ctx->hb, sizeof(double), hipMemcpyDeviceToHost, ctx->st));
        // only iteration 0 needs a value before its first trial (lambda from max diag); later
        // iterations read this iteration's chi2 together with the first trial's scalars
        bool chi_pending = true;
        if (it == 0) {
            HIPOK(hipMemcpyAsync(&head[2], B.scal + 2, sizeof(double), hipMemcpyDeviceToHost, ctx->st));
            HIPOK(hipStreamSynchronize(ctx->st));
            currentChi = head[0];
            chi_pending = false;
            R.chi2_initial = currentChi;
            lambda = prm->user_lambda > 0 ? prm->user_lambda : tau * head[2];
            ni = 2;
        }
        double rho = 0;
        int qmax = 0;
        do {
            push_state(ctx);
            hipEventRecord(ctx->ev[2], ctx->st);
            HIPOK(hipMemsetAsync(B.flag, 0, sizeof(int), ctx->st));
            ba_launch_schur(B, lambda, ctx->st);                  // setLambda; Schur complement
            if ((rc = allreduce(ctx, B.Sred, (int64_t)B.ns * (B.ns + 1) / 2 + B.ns, 0))) return rc;
            ba_launch_dense_solve(B, lambda, ctx->st);            // LinearSolverEigen on Hschur
            hipEventRecord(ctx->ev[3], ctx->st);
            ba_launch_backsub_update(B, ctx->st);                 // landmarks; _optimizer->update(x)
            hipEventRecord(ctx->ev[4], ctx->st);
            linearize(ctx, false, B.scal);                        // computeActiveErrors; activeRobustChi2
            ba_launch_scale(B, lambda, B.scal + 1, B.scal + 3, ctx->st);
            if ((rc = allreduce(ctx, B.scal, 2, 0))) return rc;
            hipEventRecord(ctx->ev[5], ctx->st);
            double *sc = ctx->hpin + 4;
            HIPOK(hipMemcpyAsync(sc, B.scal, sizeof(double) * 4, hipMemcpyDeviceToHost, ctx->st));
            HIPOK(hipMemcpyAsync(ctx->ipin, B.flag, sizeof(int), hipMemcpyDeviceToHost, ctx->st));
            HIPOK(hipStreamSynchronize(ctx->st));
            if (chi_pending) { currentChi = head[0]; chi_pending = false; }
            if (qmax == 0) t_lin += ev_ms(ctx, 0, 1);
            const int flag = *ctx->ipin;
            t_fac += ev_ms(ctx, 2, 3); t_sol += ev_ms(ctx, 3, 4); t_upd += ev_ms(ctx, 4, 5);
            const bool ok2 = flag == 0;
            const double tempChi = ok2 ? sc[0] : std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            const double scale = (sc[1] + sc[3]) + 1e-3;
            rho /= scale;
            R.trials_total++;
            if (rho > 0 && std::isfinite(tempChi) && ok2) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                lambda *= std::max(1. / 3., alpha);
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                pop_state(ctx);
                R.trials_rejected++;
            }
            qmax++;
            if (!std::isfinite(lambda)) break;
        } while (rho < 0 && qmax < max_trials);
        if (it < DEFTRI_MAX_REPORT_ITERS) { R.chi2_iter[it] = currentChi; R.trials_iter[it] = qmax; }
        if (prm->verbose)
            std::fprintf(stderr, "[deftri-ba] it %d chi2 %.9e lambda %.6e trials %d\n", it, currentChi, lambda, qmax);
        if (qmax == max_trials || rho == 0 || !std::isfinite(lambda)) { status = DEFTRI_STATUS_TERMINATE; it++; break; }
    }
    HIPOK(hipStreamSynchronize(ctx->st));
    R.chi2_final = currentChi;
    R.status = status;
    R.iterations = it;
    R.lambda_final = lambda;
    R.ms_linearize = t_lin; R.ms_factor = t_fac; R.ms_solve = t_sol; R.ms_update = t_upd;
    R.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    return 0;
}

int deftri_ba_compute_errors(deftri_ba_ctx *ctx, const uint8_t *mask) {
    if (!ctx || !ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(ctx->device);
    uint8_t *dsel = nullptr;
    if (mask && ctx->E > 0) {
        std::vector<uint8_t> sel(ctx->E);
        for (int32_t s = 0; s < ctx->E; s++) sel[s] = mask[ctx->perm[s]];
        HIPOK(hipMalloc((void **)&dsel, (size_t)ctx->E));
        HIPOK(hipMemcpy(dsel, sel.data(), (size_t)ctx->E, hipMemcpyHostToDevice));
    }
    ba_launch_edges(ctx->B, ctx->st, false, true, dsel);
    hipError_t e = hipStreamSynchronize(ctx->st);
    if (dsel) hipFree(dsel);
    HIPOK(e);
    return 0;
}

int deftri_ba_edge_chi2(deftri_ba_ctx *ctx, double *chi2, uint8_t *depth_positive) {
    if (!ctx || !ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(ctx->device);
    const int32_t E = ctx->E;
    if (E == 0) return 0;
    double *dchi = nullptr;
    uint8_t *ddp = nullptr;
    HIPOK(hipMalloc((void **)&dchi, sizeof(double) * (size_t)E));
    HIPOK(hipMalloc((void **)&ddp, (size_t)E));
    ba_launch_edge_chi2(ctx->B, ctx->d_perm, dchi, ddp, ctx->st);
    hipError_t e1 = hipSuccess, e2 = hipSuccess;
    if (chi2) e1 = hipMemcpyAsync(chi2, dchi, sizeof(double) * (size_t)E, hipMemcpyDeviceToHost, ctx->st);
    if (depth_positive) e2 = hipMemcpyAsync(depth_positive, ddp, (size_t)E, hipMemcpyDeviceToHost, ctx->st);
    hipError_t e3 = hipStreamSynchronize(ctx->st);
    hipFree(dchi);
    hipFree(ddp);
    HIPOK(e1); HIPOK(e2); HIPOK(e3);
    return 0;
}

int deftri_ba_download(deftri_ba_ctx *ctx, double *poses, double *points) {
    if (!ctx || !ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(ctx->device);
    HIPOK(hipStreamSynchronize(ctx->st));
    if (poses) HIPOK(hipMemcpy(poses, ctx->B.poses, sizeof(double) * 7 * (size_t)ctx->K, hipMemcpyDeviceToHost));
    if (points) HIPOK(hipMemcpy(points, ctx->B.points, sizeof(double) * 3 * (size_t)ctx->P, hipMemcpyDeviceToHost));
    return 0;
}

int deftri_ba_eval_system(deftri_ba_ctx *ctx, int32_t level, double lambda, double *chi2, double *S, double *rhs,
                          double *dx, double *b, int32_t *ns_out) {
    if (!ctx || !ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(ctx->device);
    int rc = prepare_active(ctx, level);
    if (rc) return rc;
    BADev &B = ctx->B;
    const int32_t K = ctx->K, P = ctx->P, ns = B.ns;
    linearize(ctx, true, ctx->hb);
    if ((rc = allreduce(ctx, ctx->hb, 1 + 42 * (int64_t)K, 0))) return rc;
    HIPOK(hipMemsetAsync(B.flag, 0, sizeof(int), ctx->st));
    ba_launch_schur(B, lambda, ctx->st);
    const int64_t NE = (int64_t)ns * (ns + 1) / 2 + ns;
    if ((rc = allreduce(ctx, B.Sred, NE, 0))) return rc;
    ba_launch_dense_solve(B, lambda, ctx->st);
    if (P > 0 || K > 0) {                                         // backsub writes dxl; undo the update
        push_state(ctx);
        ba_launch_backsub_update(B, ctx->st);
        pop_state(ctx);
    }
    std::vector<double> hb(1 + 42 * (size_t)K), sred(NE), dxp(6 * (size_t)K), dxl(3 * (size_t)P), bl(3 * (size_t)P);
    std::vector<int32_t> sidx(K);
    std::vector<uint8_t> pfree(P);
    HIPOK(hipMemcpyAsync(hb.data(), ctx->hb, sizeof(double) * hb.size(), hipMemcpyDeviceToHost, ctx->st));
    if (NE) HIPOK(hipMemcpyAsync(sred.data(), B.Sred, sizeof(double) * NE, hipMemcpyDeviceToHost, ctx->st));
    if (K) HIPOK(hipMemcpyAsync(dxp.data(), B.dxp, sizeof(double) * dxp.size(), hipMemcpyDeviceToHost, ctx->st));
    if (K) HIPOK(hipMemcpyAsync(sidx.data(), B.pose_sidx, sizeof(int32_t) * K, hipMemcpyDeviceToHost, ctx->st));
    if (P) {
        HIPOK(hipMemcpyAsync(dxl.data(), B.dxl, sizeof(double) * dxl.size(), hipMemcpyDeviceToHost, ctx->st));
        HIPOK(hipMemcpyAsync(bl.data(), B.bl, sizeof(double) * bl.size(), hipMemcpyDeviceToHost, ctx->st));
        HIPOK(hipMemcpyAsync(pfree.data(), B.pt_free, P, hipMemcpyDeviceToHost, ctx->st));
    }
    HIPOK(hipStreamSynchronize(ctx->st));
    // ba_launch_backsub_update + pop restored the state but not the cached errors: recompute them
    ba_launch_edges(B, ctx->st, false, false);
    HIPOK(hipStreamSynchronize(ctx->st));
    if (ns_out) *ns_out = ns;
    if (chi2) *chi2 = hb[0];
    const double *Hpp = hb.data() + 1, *bp = hb.data() + 1 + 36 * (size_t)K;
    std::vector<int32_t> spose(B.nfree);
    for (int32_t k = 0; k < K; k++) if (sidx[k] >= 0) spose[sidx[k]] = k;
    const int64_t ntri = (int64_t)ns * (ns + 1) / 2;
    if (S) {
        for (int32_t r = 0; r < ns; r++)
            for (int32_t c = 0; c <= r; c++) {
                double h = sred[(int64_t)r * (r + 1) / 2 + c];
                if (r / 6 == c / 6) h = Hpp[36 * spose[r / 6] + 6 * (r % 6) + (c % 6)] + h;
                if (r == c) h = (Hpp[36 * spose[r / 6] + 7 * (r % 6)] + lambda) + sred[(int64_t)r * (r + 1) / 2 + c];
                S[(int64_t)r * ns + c] = h;
                S[(int64_t)c * ns + r] = h;
            }
    }
    if (rhs)
        for (int32_t r = 0; r < ns; r++) rhs[r] = bp[6 * spose[r / 6] + r % 6] + sred[ntri + r];
    if (dx) {
        std::memcpy(dx, dxp.data(), sizeof(double) * dxp.size());
        for (int32_t l = 0; l < P; l++)
            for (int c = 0; c < 3; c++) dx[6 * (int64_t)K + 3 * l + c] = pfree[l] ? dxl[3 * (size_t)l + c] : 0.0;
    }
    if (b) {
        for (int32_t k = 0; k < K; k++)
            for (int c = 0; c < 6; c++) b[6 * k + c] = sidx[k] >= 0 ? bp[6 * k + c] : 0.0;
        for (int32_t l = 0; l < P; l++)
            for (int c = 0; c < 3; c++) b[6 * (int64_t)K + 3 * l + c] = pfree[l] ? bl[3 * (size_t)l + c] : 0.0;
    }
    return 0;
}

int deftri_rccl_unique_id(uint8_t id[128]) {
    if (!id) return DEFTRI_E_ARG;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return DEFTRI_E_HIP;
    std::memcpy(id, &u, 128);
    return 0;
}

int deftri_ba_dist_init_rccl(deftri_ba_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t id[128]) {
    if (!ctx || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !id)) return DEFTRI_E_ARG;
    hipSetDevice(ctx->device);
    if (ctx->comm) { ncclCommDestroy(ctx->comm); ctx->comm = nullptr; }
    ctx->fn = nullptr;
    ctx->nranks = nranks; ctx->rank = rank;
    if (!id) return 0;                        // one rank without RCCL
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    ncclResult_t r = ncclCommInitRank(&ctx->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        ctx->comm = nullptr; ctx->nranks = 1; ctx->rank = 0;
        return fail(ctx, DEFTRI_E_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    return 0;
}

int deftri_ba_dist_set_allreduce(deftri_ba_ctx *ctx, int32_t nranks, int32_t rank, deftri_allreduce_fn fn,
                                 void *user) {
    if (!ctx || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !fn)) return DEFTRI_E_ARG;
    if (ctx->comm) { ncclCommDestroy(ctx->comm); ctx->comm = nullptr; }
    ctx->nranks = nranks; ctx->rank = rank;
    ctx->fn = nranks > 1 ? fn : nullptr;
    ctx->fn_user = user;
    return 0;
}

int deftri_ba_profile_trial(deftri_ba_ctx *ctx, double lambda, deftri_kernel_stat *stats, int32_t max_stats,
                            int32_t *n_stats) {
    if (!ctx || !stats || !n_stats) return DEFTRI_E_ARG;
    if (!ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(ctx->device);
    int rc = prepare_active(ctx, 0);
    if (rc) return rc;
    BADev &B = ctx->B;
    KProf prof;
    ba_set_profiler(&prof);
    set_profiler(&prof);
    linearize(ctx, true, ctx->hb);
    push_state(ctx);
    ba_launch_schur(B, lambda, ctx->st);
    ba_launch_dense_solve(B, lambda, ctx->st);
    ba_launch_backsub_update(B, ctx->st);
    linearize(ctx, false, B.scal);
    ba_launch_scale(B, lambda, B.scal + 1, B.scal + 3, ctx->st);
    pop_state(ctx);
    set_profiler(nullptr);
    ba_set_profiler(nullptr);
    HIPOK(hipStreamSynchronize(ctx->st));
    int32_t n = 0;
    for (const auto &r : prof.recs) {
        float ms = 0;
        hipEventElapsedTime(&ms, r.e0, r.e1);
        int32_t k = 0;
        for (; k < n; k++) if (std::strcmp(stats[k].name, r.name) == 0) break;
        if (k == n) {
            if (n >= max_stats) continue;
            std::memset(&stats[n], 0, sizeof(stats[n]));
            std::strncpy(stats[n].name, r.name, sizeof(stats[n].name) - 1);
            n++;
        }
        stats[k].launches++;
        stats[k].ms += ms;
    }
    for (int32_t k = 0; k < n; k++) {
        // edge ids 8, obs 16, info 8, flags 2, point gather 24; err 16, chi2 8+8, w 8, omega_r 16, J 48+96
        // (the with-Jacobian launch; the chi2-only launch writes 32 B of the 200)
        if (!std::strcmp(stats[k].name, "ba_edges")) stats[k].bytes = (double)B.E * ((58 + 200) + (58 + 32));
        if (!std::strcmp(stats[k].name, "ba_dense_ldlt")) stats[k].flops = (double)B.ns * B.ns * B.ns / 3.0;
    }
    for (hipEvent_t e : prof.pool) hipEventDestroy(e);
    *n_stats = n;
    return 0;
}

}  // extern "C"
