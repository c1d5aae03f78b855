// solver.cpp — C-ABI (include/deftri.h): context, upload, g2o-semantics Levenberg–Marquardt on
// the device, download, diagnostics.  The LM control flow restates g2o's
// OptimizationAlgorithmLevenberg::solve + SparseOptimizer::optimize as driven by the reference's
// `optimizer.optimize(nOptIterations)` (Modules/Optimization/g2oBundleAdjustment.cc:959-962):
//   per iteration: computeActiveErrors, activeRobustChi2, buildSystem, lambda init (it 0:
//   tau * max diag H), then trials { push; setLambda; solve; update; restoreDiagonal;
//   computeActiveErrors; rho = (chi_cur - chi_new) / (dx.(lambda dx + b) + 1e-3); accept
//   (lambda *= max(1/3, min(2/3, 1-(2rho-1)^3)), ni = 2) or reject (lambda *= ni, ni *= 2, pop) }
//   while rho < 0 && trials < maxTrials; Terminate if trials == maxTrials || rho == 0 || !finite(lambda).
// Every arithmetic step runs on the GPU; the host only reads back the three scalars the control
// flow branches on (chi2_new, dx.(lambda dx + b), zero-pivot flag) once per trial.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <string>
#include <thread>
#include <vector>

#include <memory>

#include "../../include/deftri.h"
#include "graph_builder.h"
#include "kernels.h"
#include "pcg.h"
#include "spcg.h"
#include "exit_guard.h"
#include "symbolic.h"

using namespace deftri;

namespace deftri {
int plan_emulate_solve(const Symbolic &S, const double *H, double lambda, const double *rhs, double *x,
                       const std::function<int(int, int, double *, int64_t)> *xfer = nullptr,
                       const double *bpart = nullptr);
}

namespace {

constexpr int kRedParts = 512;
constexpr double kPcgDefaultTol = 1e-12;    // relative residual ||b - A x|| / ||b||
constexpr int kPcgDefaultMaxIt = 200;     // before a plan is uploaded
constexpr int kPcgMaxIt = 4096;
constexpr int64_t kIterativeMinUnknowns = 50000;   // DEFTRI_PLAN_AUTO: the iterative plan from here up

struct HostProblem {
    deftri_problem_desc d{};
    std::vector<double> points, tg, scales, cam_pose, rep_obs, rep_info, dep_meas, dep_info, arap_w, rot,
        pair_area, pair_info, order_xy;
    std::vector<float> cam_kb8;
    std::vector<int32_t> rep_point, rep_cam, dep_point, dep_scale, dep_cam, arap_pts, arap_pair, arap_rot;
};

template <class T>
static void cp(std::vector<T> &v, const T *p, int64_t n) {
    v.assign(p ? p : nullptr, p ? p + n : nullptr);
    if (!p) v.clear();
}

static void quat_norm(double *q) {      // SE3Quat::normalizeRotation
    if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
    double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int k = 0; k < 4; k++) q[k] /= n;
}

static void quat_mat(const double *q, double *R) {
    double x = q[0], y = q[1], z = q[2], w = q[3];
    double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    double twx = tx * w, twy = ty * w, twz = tz * w;
    double txx = tx * x, txy = ty * x, txz = tz * x;
    double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

}  // namespace

// Speculative LM trials ("lambda lanes").  g2o's trial sequence inside an iteration is fixed in
// advance: trial q uses lambda_q, and a rejection sets lambda_{q+1} = lambda_q * ni_q,
// ni_{q+1} = 2 ni_q.  A round factors and solves the next nl trials in ONE batched pass: every
// factor/solve launch carries the lanes in blockIdx.y, each lane with its own arena, panel inverses,
// solve vectors and dx (DevPlan::lo strides), so the latency-bound panel chain is paid once for nl
// trials.  Each lane's update then goes to a scratch copy of the state where its chi2 is evaluated;
// the host replays the accept/reject sequence in trial order.  Every lane computes exactly the
// numbers the sequential loop would (same kernels, same order of operations, no atomics).
// default lanes: 2 while a factorization is latency-bound (measured ms/iteration over 25 LM
// iterations, 1 -> 2 lanes: 1k corr. 1.93 -> 1.46, 10k 5.08 -> 4.51, 30k 9.86 -> 8.45), 1 once the
// big trailing updates saturate the MFMA pipes (100k / C2: 23.2 -> 25.4, a 3-lane round costs 2.1
// trials); the switch sits between 30k (~13 GFLOP per factorization) and C2 (80 GFLOP)
constexpr double kLaneFlopLimit = 3e10;
struct Lane {
    DevProblem P;         // points / scales / tg / chi_* are the lane's scratch; the rest is shared
    double *part = nullptr, *scal = nullptr;   // scal: [0] chi2 [1] scale [4..6] partial chi2
};

struct deftri_ctx {
    int device = 0;
    hipStream_t st = nullptr;
    hipStream_t side = nullptr;                 // trailing "rest" updates overlapping the panel chain
    hipEvent_t sync_ev[64]{};                   // cross-stream ordering events (timing disabled)
    std::string err;
    bool have = false;        // uploaded to the device
    bool analysed = false;    // symbolic plan available
    HostProblem hp;
    Symbolic S;
    DevProblem P;
    DevPlan L;
    std::vector<void *> allocs;
    double *d_dx = nullptr, *d_part = nullptr, *d_scal = nullptr;   // d_scal: [0]=chi2 [1]=scale [2]=maxdiag
    double *hpin = nullptr;                 // pinned host staging of the per-trial scalars (32 doubles; [16..23] PCG record)
    int *ipin = nullptr;                    // pinned host staging of the zero-pivot flag
    std::vector<double *> init_state;       // device copies of the initial state
    hipEvent_t ev[8]{};
    // map-level graph (deftri_arap_build_graph)
    GraphResult graph;
    std::unique_ptr<GraphDevice> gdev;      // computeR on this context's device (graph_dev.hip)
    // speculative lambda lanes (see Lane)
    int analytic_jac = 0;                   // deftri_arap_optimization: 0 g2o numeric (reference), 1 analytic
    bool prof_analytic = false;             // deftri_profile_trial linearizes like the last solve_lm
    int max_lanes = 0;                      // 0: default (DEFTRI_LM_LANES, else by factorization size)
    int f32_update = 0;                     // deftri_set_factor_precision
    std::vector<Lane> lanes;                // device buffers: per uploaded problem
    DevPlan LB;                             // batched plan view: lanes' arenas / inverses / vectors / flags
    double *dx_lanes = nullptr;             // [lane][ndof]
    double *lane_pin = nullptr;             // pinned: [2t] chi2_new, [2t+1] dx.(lambda dx + b)
    int *lane_ipin = nullptr;               // pinned: zero-pivot flag per lane
    // point-sharded plan (DistPlan, symbolic.h): this context is rank `rank` of `nranks`; transfers
    // and all-reduces go through RCCL on the solver stream or through a caller-supplied host callback
    int rank = 0, nranks = 1;
    ncclComm_t comm = nullptr;
    deftri_xfer_fn xfn = nullptr;
    void *xuser = nullptr;
    std::vector<double> xstage;             // host staging of the callback transport
    HostProblem hloc;                       // the rank's problem: full state, owned edges only
    double *d_xbuf = nullptr;               // staging of the rank's transfers (DistPlan::Xfer::buf_off)
    double *d_diagv = nullptr;              // diag(H) partials (lambda init)
    double *d_dofw = nullptr;               // 1 on the dofs of this rank's fronts
    double *hook_x = nullptr;               // solution vector of the solve in flight (backward transfers)
    int hook_rc = 0;                        // first transport error inside a level hook
    bool dist() const { return nranks > 1; }
    uint64_t plan_hash = 0;                 // structure_hash of the analysed problem
    int64_t plan_reuses = 0;                // uploads that reused the plan (values only)
    // one sequential trial's device work (setLambda scatter + factorization + solve: ~500 launches
    // at C2) captured once per uploaded plan and replayed as one graph launch; lambda travels through
    // d_lam.  Built lazily; dropped with the device buffers.
    hipGraphExec_t trial_graph = nullptr;
    bool trial_graph_failed = false;
    double *d_lam = nullptr;
    // LM step by block-Jacobi PCG (pcg.h) with the factorization as the fallback
    int lin_solver = DEFTRI_SOLVER_PCG;     // deftri_set_linear_solver
    double pcg_tol = kPcgDefaultTol;
    int pcg_max_it = 0;                     // 0: pcg_auto_it
    bool pcg_avail = false;                 // single-rank plan with a row view on the device
    std::string pcg_why;                    // why not (or why not matrix-free), when not
    bool pcg_mf = false;                    // the matrix-free product (pcg.h)
    PcgDev G;
    double pcg_bytes = 0, pcg_flops = 0;    // per product launch (profile_trial roofline)
    int pcg_auto_it = kPcgDefaultMaxIt;     // default budget of the uploaded plan (cost model)
    int pcg_last_its = 8;                   // iterations of the last converged solve (first chunk size)
    int pcg_step_its = 0, pcg_step_solved = 0;   // the last PCG step (deftri_last_step_info)
    bool pcg_packed = false;                // sliced blocks repacked from the current assembly
    bool assembled = false;                 // L.hval / L.b hold the current linearization's H, b
    // the point-sharded iterative plan (spcg.h; deftri_set_plan): when sp_on, every solve entry point
    // runs on `sp` and no multifrontal plan exists
    int plan_mode = DEFTRI_PLAN_AUTO;
    int jac_fp32 = 0;                       // deftri_set_jacobian_storage
    std::unique_ptr<SpSolver> sp;
    std::thread sp_reaper;                  // a re-upload's previous solver, destroyed off the caller's thread
    bool sp_on = false;
    SpTransport *sp_tr = nullptr;           // RCCL / callback transport of `sp` (owned)
    int small_direct = 0;                   // PCG skipped for this problem (too small to win, see upload)
    int pair_window = 0;                    // deftri_set_pair_window (graph builds)
};

namespace {

int fail(deftri_ctx *c, int code, const std::string &m) {
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
int dalloc(deftri_ctx *ctx, T **p, int64_t n) {
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
int dput(deftri_ctx *ctx, T **p, const T *h, int64_t n) {
    int rc = dalloc(ctx, p, n);
    if (rc) return rc;
    if (n > 0 && h) HIPOK(hipMemcpy(*p, h, sizeof(T) * (size_t)n, hipMemcpyHostToDevice));
    return 0;
}

template <class T>
int dput(deftri_ctx *ctx, T **p, const std::vector<T> &v) { return dput(ctx, p, v.data(), (int64_t)v.size()); }

void drop_trial_graph(deftri_ctx *ctx) {
    if (ctx->trial_graph) hipGraphExecDestroy(ctx->trial_graph);
    ctx->trial_graph = nullptr;
    ctx->trial_graph_failed = false;
}

void join_reaper(deftri_ctx *ctx) {
    if (ctx->sp_reaper.joinable()) ctx->sp_reaper.join();
}

// reap_async (an iterative re-upload): the previous solver's streams, events, pinned and device
// buffers are released on a thread of their own while the caller builds the next plan on the host
// (~10 ms of hipFree / hipHostFree at C2); the new solver joins it before its first allocation, and
// every other free_device (context destroy included) joins it first
void free_device(deftri_ctx *ctx, bool reap_async = false) {
    join_reaper(ctx);
    if (reap_async && ctx->sp) {
        SpSolver *old = ctx->sp.release();
        const int dev = ctx->device;
        ctx->sp_reaper = std::thread([old, dev] {
            hipSetDevice(dev);
            delete old;
        });
    }
    ctx->sp.reset();
    ctx->sp_on = false;
    drop_trial_graph(ctx);
    for (void *p : ctx->allocs) hipFree(p);
    ctx->allocs.clear();
    ctx->P = DevProblem();
    ctx->L = DevPlan();
    ctx->lanes.clear();
    ctx->LB = DevPlan();
    ctx->dx_lanes = nullptr;
    ctx->init_state.clear();
    ctx->have = false;
}

int validate(deftri_ctx *ctx, const deftri_problem_desc *d) {
    if (!d) return fail(ctx, DEFTRI_E_ARG, "null descriptor");
    if (d->n_points < 0 || d->n_pairs < 0 || d->n_scales < 0 || d->n_cams < 0 || d->n_rep < 0 || d->n_depth < 0 ||
        d->n_arap < 0 || d->n_rot < 0)
        return fail(ctx, DEFTRI_E_ARG, "negative count");
    auto need = [&](const void *p, int64_t n, const char *nm) -> bool {
        if (n > 0 && !p) { ctx->err = std::string("missing array ") + nm; return false; }
        return true;
    };
    if (!need(d->points, d->n_points, "points") || !need(d->tg, d->n_pairs, "tg") ||
        !need(d->scales, d->n_scales, "scales") || !need(d->cam_kb8, d->n_cams, "cam_kb8") ||
        !need(d->cam_pose, d->n_cams, "cam_pose") || !need(d->rep_point, d->n_rep, "rep_point") ||
        !need(d->rep_cam, d->n_rep, "rep_cam") || !need(d->rep_obs, d->n_rep, "rep_obs") ||
        !need(d->rep_info, d->n_rep, "rep_info") || !need(d->dep_point, d->n_depth, "dep_point") ||
        !need(d->dep_scale, d->n_depth, "dep_scale") || !need(d->dep_cam, d->n_depth, "dep_cam") ||
        !need(d->dep_meas, d->n_depth, "dep_meas") || !need(d->dep_info, d->n_depth, "dep_info") ||
        !need(d->arap_pts, d->n_arap, "arap_pts") || !need(d->arap_pair, d->n_arap, "arap_pair") ||
        !need(d->arap_rot, d->n_arap, "arap_rot") || !need(d->arap_w, d->n_arap, "arap_w") ||
        !need(d->rot, d->n_rot, "rot") || !need(d->pair_area, d->n_pairs, "pair_area") ||
        !need(d->pair_info, d->n_pairs, "pair_info"))
        return DEFTRI_E_ARG;
    auto in = [](int64_t v, int64_t hi) { return v >= 0 && v < hi; };
    for (int e = 0; e < d->n_rep; e++)
        if (!in(d->rep_point[e], d->n_points) || !in(d->rep_cam[e], d->n_cams))
            return fail(ctx, DEFTRI_E_ARG, "reprojection edge " + std::to_string(e) + ": index out of range");
    for (int e = 0; e < d->n_depth; e++)
        if (!in(d->dep_point[e], d->n_points) || !in(d->dep_scale[e], d->n_scales) || !in(d->dep_cam[e], d->n_cams))
            return fail(ctx, DEFTRI_E_ARG, "depth edge " + std::to_string(e) + ": index out of range");
    for (int e = 0; e < d->n_arap; e++) {
        const int32_t *v = d->arap_pts + 4 * (int64_t)e;
        for (int k = 0; k < 4; k++)
            if (!in(v[k], d->n_points)) return fail(ctx, DEFTRI_E_ARG, "ARAP edge " + std::to_string(e) + ": point index out of range");
        for (int a = 0; a < 4; a++)
            for (int b = a + 1; b < 4; b++)
                if (v[a] == v[b]) return fail(ctx, DEFTRI_E_ARG, "ARAP edge " + std::to_string(e) + ": repeated vertex");
        if (!in(d->arap_pair[e], d->n_pairs) || !in(d->arap_rot[2 * (int64_t)e], d->n_rot) ||
            !in(d->arap_rot[2 * (int64_t)e + 1], d->n_rot))
            return fail(ctx, DEFTRI_E_ARG, "ARAP edge " + std::to_string(e) + ": pair/rotation index out of range");
    }
    for (int64_t i = 0; i < 3 * (int64_t)d->n_points; i++)
        if (!std::isfinite(d->points[i])) return fail(ctx, DEFTRI_E_ARG, "non-finite point coordinate");
    return 0;
}

void copy_host(HostProblem &h, const deftri_problem_desc *d) {
    int64_t P = d->n_points, Q = d->n_pairs, S = d->n_scales, C = d->n_cams, R = d->n_rep, D = d->n_depth,
            E = d->n_arap, NR = d->n_rot;
    cp(h.points, d->points, 3 * P); cp(h.tg, d->tg, 7 * Q); cp(h.scales, d->scales, S);
    cp(h.cam_kb8, d->cam_kb8, 8 * C); cp(h.cam_pose, d->cam_pose, 7 * C);
    cp(h.rep_point, d->rep_point, R); cp(h.rep_cam, d->rep_cam, R); cp(h.rep_obs, d->rep_obs, 2 * R);
    cp(h.rep_info, d->rep_info, R);
    cp(h.dep_point, d->dep_point, D); cp(h.dep_scale, d->dep_scale, D); cp(h.dep_cam, d->dep_cam, D);
    cp(h.dep_meas, d->dep_meas, D); cp(h.dep_info, d->dep_info, D);
    cp(h.arap_pts, d->arap_pts, 4 * E); cp(h.arap_pair, d->arap_pair, E); cp(h.arap_rot, d->arap_rot, 2 * E);
    cp(h.arap_w, d->arap_w, E); cp(h.rot, d->rot, 9 * NR); cp(h.pair_area, d->pair_area, Q);
    cp(h.pair_info, d->pair_info, Q);
    cp(h.order_xy, d->order_xy, d->order_xy ? 2 * P : 0);
    for (int64_t q = 0; q < Q; q++) quat_norm(&h.tg[7 * q]);        // SE3Quat(q, t) normalizes
    for (int64_t c = 0; c < C; c++) quat_norm(&h.cam_pose[7 * c]);
    h.d = *d;
    h.d.points = h.points.data(); h.d.tg = h.tg.data(); h.d.scales = h.scales.data();
    h.d.cam_kb8 = h.cam_kb8.data(); h.d.cam_pose = h.cam_pose.data();
    h.d.rep_point = h.rep_point.data(); h.d.rep_cam = h.rep_cam.data(); h.d.rep_obs = h.rep_obs.data();
    h.d.rep_info = h.rep_info.data();
    h.d.dep_point = h.dep_point.data(); h.d.dep_scale = h.dep_scale.data(); h.d.dep_cam = h.dep_cam.data();
    h.d.dep_meas = h.dep_meas.data(); h.d.dep_info = h.dep_info.data();
    h.d.arap_pts = h.arap_pts.data(); h.d.arap_pair = h.arap_pair.data(); h.d.arap_rot = h.arap_rot.data();
    h.d.arap_w = h.arap_w.data(); h.d.rot = h.rot.data(); h.d.pair_area = h.pair_area.data();
    h.d.pair_info = h.pair_info.data();
    h.d.order_xy = h.order_xy.empty() ? nullptr : h.order_xy.data();
}

// Structure of the normal equations: the counts and every index array (what Eigen's AMD ordering
// and the symbolic analysis see).  Two problems with the same hash share the plan: NLopt's
// outerObjective evaluations (nloptOptimization.cc:4-37) rebuild the same graph on clones of one
// map with other weights, so every evaluation after the first reuses the analysis and the device
// plan and only copies the values.
uint64_t structure_hash(const deftri_problem_desc &d) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void *p, size_t n) {      // 8 bytes per step (a pre-filter, see same_structure)
        const unsigned char *b = (const unsigned char *)p;
        size_t i = 0;
        for (; i + 8 <= n; i += 8) {
            uint64_t w;
            std::memcpy(&w, b + i, 8);
            h = (h ^ w) * 0x9E3779B97F4A7C15ull;
            h ^= h >> 29;
        }
        for (; i < n; i++) { h ^= b[i]; h *= 1099511628211ull; }
    };
    const int32_t cnt[8] = {d.n_points, d.n_pairs, d.n_scales, d.n_cams, d.n_rep, d.n_depth, d.n_arap, d.n_rot};
    mix(cnt, sizeof(cnt));
    mix(d.rep_point, sizeof(int32_t) * (size_t)d.n_rep);
    mix(d.rep_cam, sizeof(int32_t) * (size_t)d.n_rep);
    mix(d.dep_point, sizeof(int32_t) * (size_t)d.n_depth);
    mix(d.dep_scale, sizeof(int32_t) * (size_t)d.n_depth);
    mix(d.dep_cam, sizeof(int32_t) * (size_t)d.n_depth);
    mix(d.arap_pts, sizeof(int32_t) * 4 * (size_t)d.n_arap);
    mix(d.arap_pair, sizeof(int32_t) * (size_t)d.n_arap);
    mix(d.arap_rot, sizeof(int32_t) * 2 * (size_t)d.n_arap);
    return h;
}

// the hash is only a pre-filter: the counts and every index array must match exactly before a plan is
// reused (a collision would scatter H into the wrong blocks)
bool same_structure(const deftri_problem_desc &a, const deftri_problem_desc &b) {
    if (a.n_points != b.n_points || a.n_pairs != b.n_pairs || a.n_scales != b.n_scales || a.n_cams != b.n_cams ||
        a.n_rep != b.n_rep || a.n_depth != b.n_depth || a.n_arap != b.n_arap || a.n_rot != b.n_rot)
        return false;
    auto eq = [](const int32_t *x, const int32_t *y, int64_t n) {
        return n == 0 || (x && y && std::memcmp(x, y, sizeof(int32_t) * (size_t)n) == 0);
    };
    return eq(a.rep_point, b.rep_point, a.n_rep) && eq(a.rep_cam, b.rep_cam, a.n_rep) &&
           eq(a.dep_point, b.dep_point, a.n_depth) && eq(a.dep_scale, b.dep_scale, a.n_depth) &&
           eq(a.dep_cam, b.dep_cam, a.n_depth) && eq(a.arap_pts, b.arap_pts, 4 * (int64_t)a.n_arap) &&
           eq(a.arap_pair, b.arap_pair, a.n_arap) && eq(a.arap_rot, b.arap_rot, 2 * (int64_t)a.n_arap);
}

// the coordinates the row order is derived from (order_xy, else the points' x, y): equal on both
// problems for the iterative plan to be reused
bool same_order_coordinates(const deftri_problem_desc &a, const deftri_problem_desc &b) {
    if (a.n_points != b.n_points || (a.order_xy == nullptr) != (b.order_xy == nullptr)) return false;
    if (a.order_xy) return std::memcmp(a.order_xy, b.order_xy, sizeof(double) * 2 * (size_t)a.n_points) == 0;
    return std::memcmp(a.points, b.points, sizeof(double) * 3 * (size_t)a.n_points) == 0;
}

// same structure as the uploaded plan: copy the values (state, cameras, measurements, weights,
// rotations) into the existing device buffers
int refresh_values(deftri_ctx *ctx, const HostProblem &h) {
    DevProblem &P = ctx->P;
    auto put = [&](auto *dst, const auto &v) -> hipError_t {
        return v.empty() ? hipSuccess : hipMemcpy(dst, v.data(), sizeof(v[0]) * v.size(), hipMemcpyHostToDevice);
    };
    std::vector<double> camR(9 * (size_t)std::max(P.C, 1));
    for (int c = 0; c < P.C; c++) quat_mat(&h.cam_pose[7 * c], &camR[9 * c]);
    HIPOK(put(P.points, h.points)); HIPOK(put(P.scales, h.scales)); HIPOK(put(P.tg, h.tg));
    HIPOK(put(ctx->init_state[0], h.points)); HIPOK(put(ctx->init_state[1], h.scales));
    HIPOK(put(ctx->init_state[2], h.tg));
    HIPOK(put(P.cam_kb8, h.cam_kb8)); HIPOK(put(P.cam_pose, h.cam_pose)); HIPOK(put(P.cam_R, camR));
    HIPOK(put(P.rep_obs, h.rep_obs)); HIPOK(put(P.rep_info, h.rep_info));
    HIPOK(put(P.dep_meas, h.dep_meas)); HIPOK(put(P.dep_info, h.dep_info));
    HIPOK(put(P.arap_w, h.arap_w)); HIPOK(put(P.rot, h.rot));
    HIPOK(put(P.pair_area, h.pair_area)); HIPOK(put(P.pair_info, h.pair_info));
    P.huber_delta = h.d.huber_delta;
    return 0;
}

bool mf_wanted() {
    static const bool on = [] { const char *e = std::getenv("DEFTRI_PCG_MF"); return !e || std::atoi(e) != 0; }();
    return on;
}

// the PCG budget: CG iterations that cost about one factorization + substitution, from plan sizes
// only (deterministic: the same problem always takes the same path).  Rates measured at C2: the
// LDL^T trial ~7 TF/s + ~50 us per tree level, a CG iteration ~2 TB/s of its product's bytes + ~15 us
// of launch latency, plus a quarter of a host round trip (~40 us; pcg_poll reads the record every
// 4 iterations once the predicted count is exceeded)
int pcg_budget(const Symbolic &S, double product_bytes) {
    const double t_fac = S.factor_flops / 7e9 + 0.05 * S.nlevels;   // ms
    const double t_it = product_bytes / 2e9 + 0.015 + 0.04 / 4;
    return (int)std::min<double>(kPcgMaxIt, std::max(8.0, std::ceil(t_fac / t_it)));
}

// the matrix-free PCG plan on the device (single-rank); 0 when available, else ctx->pcg_why says why
int upload_pcg_mf(deftri_ctx *ctx, const HostProblem &h) {
    const Symbolic &S = ctx->S;
    const deftri_problem_desc &d = h.d;
    const DevProblem &P = ctx->P;
    PcgMfHost mh;
    std::string why;
    if (!build_pcg_mf(S.nv, S.voff, S.vdim, S.elim_pos, d.n_pairs, d.n_scales, d.n_rep, d.n_depth, d.n_arap,
                      h.rep_point.data(), h.dep_point.data(), h.dep_scale.data(), h.arap_pts.data(),
                      h.arap_pair.data(), mh, why)) {
        ctx->pcg_why = "matrix-free plan: " + why;
        return -1;
    }
    int rc;
#define PUT(dst, src) if ((rc = dput(ctx, &(dst), src))) return rc
    PcgDev &G = ctx->G;
    G = PcgDev();
    G.mf = 1;
    G.mf_lds = std::max(mh.max_lds, 1);
    G.nv = S.nv; G.ndof = S.ndof;
    G.nheavy = (int32_t)mh.heavy_v.size();
    G.nheavy_dofs = mh.h_dofbase.back();
    G.nsl = (int32_t)mh.le_n.size();
    G.nA_sl = G.nsl;
    G.nB = (int32_t)((S.nv + 255) / 256);
    int32_t *hv, *hdb, *vh, *hf, *sv, *len, *lena, *inn, *inc, *inc2, *shn, *hshk, *ad, *atd, *rd, *dd;
    int64_t *mo, *leo, *le, *ino, *shoff, *hvb, *hvs;
    PUT(hv, mh.heavy_v); PUT(hdb, mh.h_dofbase); PUT(vh, mh.v_heavy); PUT(hf, mh.h_first); PUT(mo, mh.moff);
    PUT(sv, mh.sl_v); PUT(leo, mh.le_off); PUT(len, mh.le_n); PUT(lena, mh.le_na); PUT(le, mh.le);
    PUT(ino, mh.in_off); PUT(inn, mh.in_n); PUT(inc, mh.inc); PUT(inc2, mh.inc2);
    PUT(shn, mh.sl_hn); PUT(hshk, mh.hs_hk); PUT(shoff, mh.sl_hoff); PUT(hvb, mh.hv_slot_begin); PUT(hvs, mh.hs_pos);
    PUT(ad, mh.adof); PUT(atd, mh.atdof); PUT(rd, mh.rdof); PUT(dd, mh.ddof);
    int32_t *snt, *own_n, *own;
    int64_t *own_off;
    PUT(snt, mh.sl_nt); PUT(own_n, mh.own_n); PUT(own, mh.own); PUT(own_off, mh.own_off);
    G.mf_sl_nt = snt; G.mf_own_n = own_n; G.mf_own = own; G.mf_own_off = own_off;
    int64_t *smeta;
    int32_t *shpos;
    PUT(smeta, mh.sl_meta); PUT(shpos, mh.sl_hpos);
    G.mf_sl_meta = smeta; G.mf_sl_hpos = shpos;
#undef PUT
    G.heavy_v = hv; G.h_dofbase = hdb; G.v_heavy = vh; G.h_first = hf; G.moff = mo;
    G.sl_v = sv; G.mf_le_off = leo; G.mf_le_n = len; G.mf_le_na = lena; G.mf_le = le;
    G.mf_in_off = ino; G.mf_in_n = inn; G.mf_inc = inc; G.mf_inc2 = inc2;
    G.sl_hn = shn; G.hs_hk = hshk; G.sl_hoff = shoff; G.hv_slot_begin = hvb; G.hs_pos = hvs;
    G.nhslots = (int64_t)mh.hs_hk.size();
    G.mf_adof = ad; G.mf_atdof = atd; G.mf_rdof = rd; G.mf_ddof = dd;
    G.voff = ctx->L.voff; G.vdim = ctx->L.vdim;
    G.Jarap = P.Jarap; G.Warap = P.Warap; G.Earap = P.Earap;
    G.Jrep = P.Jrep; G.Wrep = P.Wrep; G.Erep = P.Erep;
    G.Jdep = P.Jdep; G.Wdep = P.Wdep; G.Edep = P.Edep;
    G.b = ctx->L.b;
    if ((rc = dalloc(ctx, &G.hs_part, 6 * std::max<int64_t>(G.nhslots, 1))) ||
        (rc = dalloc(ctx, &G.mf_hlin, kMfLin * std::max<int64_t>(G.nhslots, 1))) ||
        (rc = dalloc(ctx, &G.hqf, std::max(G.nheavy_dofs, 1))) || (rc = dalloc(ctx, &G.mf_diag, mh.msize)) ||
        (rc = dalloc(ctx, &G.mf_dvec, S.ndof)) || (rc = dalloc(ctx, &G.minv, mh.msize)) ||
        (rc = dalloc(ctx, &G.r, S.ndof)) || (rc = dalloc(ctx, &G.zp, 2 * S.ndof)) ||
        (rc = dalloc(ctx, &G.pq, 2 * S.ndof)) || (rc = dalloc(ctx, &G.partA, std::max(G.nA_sl, 1))) ||
        (rc = dalloc(ctx, &G.partB, 2 * (int64_t)G.nB)) || (rc = dalloc(ctx, &G.rec, (int64_t)kPcgRec * (kPcgMaxIt + 2))))
        return rc;
    ctx->pcg_avail = true;
    ctx->pcg_bytes = mh.product_bytes;
    ctx->pcg_flops = mh.product_flops;
    ctx->pcg_auto_it = pcg_budget(S, mh.product_bytes);
    return 0;
}

int upload_device(deftri_ctx *ctx, const HostProblem &h) {
    const deftri_problem_desc &d = h.d;
    DevProblem &P = ctx->P;
    P.P = d.n_points; P.Q = d.n_pairs; P.S = d.n_scales; P.C = d.n_cams;
    P.R = d.n_rep; P.D = d.n_depth; P.E = d.n_arap; P.NR = d.n_rot;
    P.huber_delta = d.huber_delta;
    int rc;
#define PUT(dst, src) if ((rc = dput(ctx, &(dst), src))) return rc
    PUT(P.points, h.points); PUT(P.scales, h.scales); PUT(P.tg, h.tg);
    if ((rc = dalloc(ctx, &P.points_bak, 3 * (int64_t)P.P))) return rc;
    if ((rc = dalloc(ctx, &P.scales_bak, P.S))) return rc;
    if ((rc = dalloc(ctx, &P.tg_bak, 7 * (int64_t)P.Q))) return rc;
    PUT(P.cam_kb8, h.cam_kb8); PUT(P.cam_pose, h.cam_pose);
    std::vector<double> camR(9 * (size_t)std::max(P.C, 1));
    for (int c = 0; c < P.C; c++) quat_mat(&h.cam_pose[7 * c], &camR[9 * c]);
    PUT(P.cam_R, camR);
    PUT(P.rep_point, h.rep_point); PUT(P.rep_cam, h.rep_cam); PUT(P.rep_obs, h.rep_obs); PUT(P.rep_info, h.rep_info);
    PUT(P.dep_point, h.dep_point); PUT(P.dep_scale, h.dep_scale); PUT(P.dep_cam, h.dep_cam);
    PUT(P.dep_meas, h.dep_meas); PUT(P.dep_info, h.dep_info);
    PUT(P.arap_pts, h.arap_pts); PUT(P.arap_pair, h.arap_pair); PUT(P.arap_rot, h.arap_rot);
    PUT(P.arap_w, h.arap_w); PUT(P.rot, h.rot); PUT(P.pair_area, h.pair_area); PUT(P.pair_info, h.pair_info);
    if ((rc = dalloc(ctx, &P.Jrep, 6 * (int64_t)P.R)) || (rc = dalloc(ctx, &P.Wrep, P.R)) ||
        (rc = dalloc(ctx, &P.Erep, 2 * (int64_t)P.R)) || (rc = dalloc(ctx, &P.chi_rep, P.R)) ||
        (rc = dalloc(ctx, &P.Jdep, 4 * (int64_t)P.D)) || (rc = dalloc(ctx, &P.Wdep, P.D)) ||
        (rc = dalloc(ctx, &P.Edep, P.D)) || (rc = dalloc(ctx, &P.chi_dep, P.D)) ||
        (rc = dalloc(ctx, &P.Jarap, 18 * (int64_t)P.E)) || (rc = dalloc(ctx, &P.Warap, P.E)) ||
        (rc = dalloc(ctx, &P.Earap, P.E)) || (rc = dalloc(ctx, &P.chi_arap, P.E)) ||
        (rc = dalloc(ctx, &P.tg_pre, 12 * 13 * (int64_t)std::max(P.Q, 1))))
        return rc;
    // keep the initial state for deftri_reset_state
    ctx->init_state.resize(3);
    if ((rc = dput(ctx, &ctx->init_state[0], h.points)) || (rc = dput(ctx, &ctx->init_state[1], h.scales)) ||
        (rc = dput(ctx, &ctx->init_state[2], h.tg)))
        return rc;

    // plan
    const Symbolic &S = ctx->S;
    DevPlan &L = ctx->L;
    L.nv = S.nv; L.ndof = S.ndof;
    PUT(L.voff, S.voff); PUT(L.vdim, S.vdim);
    L.nblocks = S.nblocks; L.hval_size = S.hval_size;
    if ((rc = dalloc(ctx, &L.hval, S.hval_size))) return rc;
    PUT(L.blk_val_off, S.blk_val_off); PUT(L.blk_arena, S.blk_arena); PUT(L.blk_rows, S.blk_rows);
    PUT(L.blk_cols, S.blk_cols); PUT(L.blk_ld, S.blk_ld); PUT(L.blk_diag, S.blk_diag);
    PUT(L.blk_row_dof, S.blk_row_dof); PUT(L.blk_col_dof, S.blk_col_dof);   // H x product, diag(H) partials
    L.nhchunks = (int64_t)S.hchunk_begin.size();
    PUT(L.hcontrib, S.hcontrib); PUT(L.hchunk_begin, S.hchunk_begin); PUT(L.hchunk_len, S.hchunk_len);
    PUT(L.hblk_chunk_begin, S.hblk_chunk_begin);
    if ((rc = dalloc(ctx, &L.hpart, 36 * L.nhchunks))) return rc;
    L.nbchunks = (int64_t)S.bchunk_begin.size();
    PUT(L.bcontrib, S.bcontrib); PUT(L.bchunk_begin, S.bchunk_begin); PUT(L.bchunk_len, S.bchunk_len);
    PUT(L.bv_chunk_begin, S.bv_chunk_begin);
    if ((rc = dalloc(ctx, &L.bpart, 6 * L.nbchunks))) return rc;
    {
        std::vector<int64_t> hh, hb;
        for (int64_t b = 0; b < S.nblocks; b++)
            if (S.hblk_chunk_begin[b + 1] - S.hblk_chunk_begin[b] > kHeavyChunks) hh.push_back(b);
        for (int64_t v = 0; v < S.nv; v++)
            if (S.bv_chunk_begin[v + 1] - S.bv_chunk_begin[v] > kHeavyChunks) hb.push_back(v);
        L.nheavy_h = (int64_t)hh.size(); L.nheavy_b = (int64_t)hb.size();
        if (!hh.empty()) PUT(L.heavy_h, hh);
        if (!hb.empty()) PUT(L.heavy_b, hb);
        if ((rc = dalloc(ctx, &L.heavy_scratch, 32 * std::max<int64_t>(36 * L.nheavy_h, 6 * L.nheavy_b)))) return rc;
    }
    if ((rc = dalloc(ctx, &L.b, S.ndof))) return rc;
    L.arena_size = S.arena_size; L.vec_size = S.vec_size;
    if ((rc = dalloc(ctx, &L.arena, S.arena_size))) return rc;
    if ((rc = dalloc(ctx, &L.vec, S.vec_size))) return rc;
    if ((rc = dalloc(ctx, &L.yvec, S.vec_size))) return rc;
    L.inv_size = S.inv_size;
    if ((rc = dalloc(ctx, &L.inv, S.inv_size))) return rc;
    {
        int32_t nf = (int32_t)S.fronts.size();
        std::vector<int32_t> m(nf), s(nf), par(nf), nch(nf), c0(nf), c1(nf), dir(nf), rb(nf), po(nf);
        std::vector<int64_t> ao(nf), vo(nf), ro(nf), bo(nf), io(nf);
        for (int32_t f = 0; f < nf; f++) {
            const Front &F = S.fronts[f];
            m[f] = F.m; s[f] = F.s; par[f] = F.parent; nch[f] = F.nchild; c0[f] = F.child[0]; c1[f] = F.child[1];
            dir[f] = F.direct; rb[f] = F.rhs_bnd; po[f] = F.panel_off;
            ao[f] = F.arena_off; vo[f] = F.vec_off; ro[f] = F.rows_off; bo[f] = F.bmap_off; io[f] = F.inv_off;
        }
        int32_t *pm, *ps, *pp, *pn, *pc0, *pc1, *pdir, *prb, *ppo, *prows, *pbmap;
        int64_t *pao, *pvo, *pro, *pbo, *pio;
        PUT(pm, m); PUT(ps, s); PUT(pp, par); PUT(pn, nch); PUT(pc0, c0); PUT(pc1, c1); PUT(pdir, dir); PUT(prb, rb); PUT(ppo, po);
        PUT(pao, ao); PUT(pvo, vo); PUT(pro, ro); PUT(pbo, bo); PUT(pio, io);
        PUT(prows, S.rows); PUT(pbmap, S.bmap);
        L.fd = FrontDev{pm, ps, pp, pn, pc0, pc1, pdir, prb, ppo, pao, pvo, pro, pbo, pio, prows, pbmap};
    }
    PUT(L.tasks, S.task_i32);
    L.levels.clear();
    for (const auto &lv : S.levels) {
        LevelDev ld{};
        for (int k = 0; k < 2; k++) { ld.ea_off[k] = lv.ea_off[k]; ld.nea[k] = lv.nea[k]; }
        for (const auto &stp : lv.steps)
            ld.steps.push_back({stp.diag_off, stp.ndiag, stp.trsm_off, stp.ntrsm, stp.upd_off, stp.nupd, stp.k0, stp.kA, stp.kmax, stp.inner, stp.stream, stp.wait_side, stp.upd_flops, stp.ntail, stp.ndiag_tail});
        ld.fwd_off = lv.fwd_off; ld.nfwd = lv.nfwd;
        for (const auto &x : lv.fsteps) ld.fsteps.push_back({x.off, x.n});
        for (const auto &x : lv.bsteps) ld.bsteps.push_back({x.off, x.n});
        ld.bgemv_off = lv.bgemv_off; ld.nbgemv = lv.nbgemv;
        ld.fchain_off = lv.fchain_off; ld.nfchain = lv.nfchain;
        ld.bchain_off = lv.bchain_off; ld.nbchain = lv.nbchain;
        L.levels.push_back(ld);
    }
    if ((rc = dalloc(ctx, &L.flag, 1))) return rc;
    if ((rc = dalloc(ctx, &ctx->d_lam, 1))) return rc;
    L.npanels = S.npanels;
    L.f32_update = ctx->f32_update;
    if ((rc = dalloc(ctx, &L.pflag, std::max<int64_t>(S.npanels, 1)))) return rc;
    HIPOK(hipMemset(L.pflag, 0, sizeof(int) * (size_t)std::max<int64_t>(S.npanels, 1)));
    if (S.trsm_fused && (rc = dalloc(ctx, &L.wbuf, 4096 * std::max<int64_t>(S.npanels, 1)))) return rc;   // else nullptr: no W
    if ((rc = dalloc(ctx, &ctx->d_dx, S.ndof))) return rc;
    HIPOK(hipMemset(ctx->d_dx, 0, sizeof(double) * (size_t)std::max<int64_t>(S.ndof, 1)));   // dofs no solve writes stay 0
    if ((rc = dalloc(ctx, &ctx->d_part, kMaxSumJobs * kRedParts))) return rc;   // launch_sum_multi: one run of parts per job
    if ((rc = dalloc(ctx, &ctx->d_scal, 8))) return rc;
    ctx->pcg_avail = false;
    ctx->pcg_why.clear();
    ctx->pcg_mf = false;
    if (ctx->dist()) {
        ctx->pcg_why = "point-sharded plan";
    } else if (mf_wanted() && upload_pcg_mf(ctx, h) == 0) {
        ctx->pcg_mf = true;                   // matrix-free product (pcg.h)
    } else {
        PcgHost ph;
        if (!build_pcg_host(S.nv, S.voff, S.vdim, S.blk_val_off, S.blk_rows, S.blk_cols, S.blk_row_dof, S.blk_col_dof,
                            S.elim_pos, ph, ctx->pcg_why)) {
            ctx->pcg_why = "row view: " + ctx->pcg_why;
        } else {
            PcgDev &G = ctx->G;
            G = PcgDev();
            G.nv = S.nv; G.ndof = S.ndof;
            G.nlight = (int32_t)ph.light_v.size();
            G.nheavy = (int32_t)ph.heavy_v.size();
            G.nhchunks = (int32_t)ph.hc_vertex.size();
            G.nheavy_dofs = ph.h_dofbase.back();
            G.nA_light = (G.nlight + 255) / 256;
            G.nsl = (int32_t)ph.sl_n.size();
            G.nA_sl = G.nsl;                  // one workgroup per slice
            G.nslots = (int64_t)ph.sl_map.size() / 64;
            G.nB = (int32_t)((S.nv + 255) / 256);
            int64_t *eb, *hb, *he, *dg, *mo;
            PcgEnt *en;
            int32_t *lv, *hv, *hcv, *hf, *hdb, *vh;
            PUT(eb, ph.ent_begin); PUT(en, ph.ent); PUT(lv, ph.light_v); PUT(hv, ph.heavy_v); PUT(hcv, ph.hc_vertex);
            PUT(hb, ph.hc_beg); PUT(he, ph.hc_end); PUT(hf, ph.h_first); PUT(hdb, ph.h_dofbase); PUT(vh, ph.v_heavy);
            PUT(dg, ph.diag_off); PUT(mo, ph.moff);
            G.ent_begin = eb; G.ent = en; G.light_v = lv; G.heavy_v = hv; G.hc_vertex = hcv; G.hc_beg = hb;
            G.hc_end = he; G.h_first = hf; G.h_dofbase = hdb; G.v_heavy = vh; G.diag_off = dg; G.moff = mo;
            G.voff = L.voff; G.vdim = L.vdim;
            {
                int32_t *sv, *sn, *snx, *scol;
                int64_t *soff, *sxoff, *smap;
                PcgEnt *sx;
                PUT(sv, ph.sl_v); PUT(sn, ph.sl_n); PUT(snx, ph.sl_nx); PUT(scol, ph.sl_col);
                PUT(soff, ph.sl_off); PUT(sxoff, ph.sl_xoff); PUT(smap, ph.sl_map); PUT(sx, ph.sl_x);
                G.sl_v = sv; G.sl_n = sn; G.sl_nx = snx; G.sl_col = scol; G.sl_off = soff; G.sl_xoff = sxoff;
                G.sl_map = smap; G.sl_x = sx;
                if ((rc = dalloc(ctx, &G.sl_val, 640 * std::max<int64_t>(G.nslots, 1)))) return rc;
                int32_t *shn, *hshk;
                int64_t *shoff, *hsmap, *hvb, *hvs;
                PcgEnt *hres;
                PUT(shn, ph.sl_hn); PUT(hshk, ph.hs_hk); PUT(shoff, ph.sl_hoff); PUT(hsmap, ph.hs_map);
                PUT(hvb, ph.hv_slot_begin); PUT(hvs, ph.hs_pos); PUT(hres, ph.hres);
                int64_t *hsvo;
                PUT(hsvo, ph.hs_voff);
                G.hs_voff = hsvo;
                G.sl_hn = shn; G.hs_hk = hshk; G.sl_hoff = shoff; G.hs_map = hsmap; G.hv_slot_begin = hvb;
                G.hs_pos = hvs; G.hres = hres;
                G.nhslots = (int64_t)ph.hs_hk.size();
                if ((rc = dalloc(ctx, &G.hs_val, std::max<int64_t>(ph.hs_size, 2))) ||
                    (rc = dalloc(ctx, &G.hs_part, 6 * std::max<int64_t>(G.nhslots, 1))) ||
                    (rc = dalloc(ctx, &G.hqf, std::max(G.nheavy_dofs, 1))))
                    return rc;
            }
            if ((rc = dalloc(ctx, &G.minv, ph.msize)) || (rc = dalloc(ctx, &G.r, S.ndof)) ||
                (rc = dalloc(ctx, &G.zp, 2 * S.ndof)) || (rc = dalloc(ctx, &G.pq, 2 * S.ndof)) ||
                (rc = dalloc(ctx, &G.partA, std::max(G.nA_sl + G.nA_light, 1))) || (rc = dalloc(ctx, &G.partB, 2 * (int64_t)G.nB)) ||
                (rc = dalloc(ctx, &G.rec, (int64_t)kPcgRec * (kPcgMaxIt + 2))))
                return rc;
            ctx->pcg_avail = true;
            const double by = ph.product_bytes, fl = ph.product_flops;
            ctx->pcg_bytes = by;
            ctx->pcg_flops = fl;
            ctx->pcg_auto_it = pcg_budget(S, by);
        }
    }
    if (std::getenv("DEFTRI_PCG_LOG"))
        std::fprintf(stderr, "[deftri] pcg: %s (budget %d)%s%s\n", !ctx->pcg_avail ? "unavailable" : ctx->pcg_mf ? "matrix-free" : "assembled",
                     ctx->pcg_auto_it, ctx->pcg_why.empty() ? "" : ": ", ctx->pcg_why.c_str());
    if (ctx->dist()) {
        if ((rc = dalloc(ctx, &ctx->d_xbuf, S.dist.xbuf_size))) return rc;
        if ((rc = dalloc(ctx, &ctx->d_diagv, S.ndof))) return rc;
        std::vector<double> w(S.dist.dof_local.begin(), S.dist.dof_local.end());
        PUT(ctx->d_dofw, w);
    }
#undef PUT
    HIPOK(hipDeviceSynchronize());
    return 0;
}

// ---- point-sharded transport ----------------------------------------------------------------
// in-place sum (op 0) / max (op 1) over the ranks of n device doubles (no-op on one rank)
int dist_allreduce(deftri_ctx *ctx, double *buf, int64_t n, int op) {
    if (!ctx->dist() || n <= 0) return 0;
    if (ctx->comm) {
        ncclResult_t r = ncclAllReduce(buf, buf, (size_t)n, ncclDouble, op == 0 ? ncclSum : ncclMax, ctx->comm, ctx->st);
        if (r != ncclSuccess) return fail(ctx, DEFTRI_E_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
        return 0;
    }
    if (!ctx->xfn) return fail(ctx, DEFTRI_E_ARG, "point-sharded context without a transport");
    if ((int64_t)ctx->xstage.size() < n) ctx->xstage.resize((size_t)n);
    HIPOK(hipMemcpyAsync(ctx->xstage.data(), buf, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, ctx->st));
    HIPOK(hipStreamSynchronize(ctx->st));
    if (ctx->xfn(ctx->xuser, op, -1, ctx->xstage.data(), n) != 0) return fail(ctx, DEFTRI_E_ARG, "all-reduce callback failed");
    HIPOK(hipMemcpyAsync(buf, ctx->xstage.data(), sizeof(double) * (size_t)n, hipMemcpyHostToDevice, ctx->st));
    return 0;
}

// point-to-point transfers of one step, in the DistPlan's global order (every rank walks the same
// list, so the host transport's blocking send/recv cannot cross); RCCL groups them
// (st: the stream the transfers are ordered on — the context's, or the iterative plan's exchange
// stream when its halo exchange runs beside the interior product)
struct P2P { int peer; bool send; double *buf; int64_t n; };
int dist_p2p(deftri_ctx *ctx, const std::vector<P2P> &ops, hipStream_t st = nullptr) {
    if (ops.empty()) return 0;
    const hipStream_t s = st ? st : ctx->st;
    if (ctx->comm) {
        ncclGroupStart();
        for (const P2P &o : ops) {
            ncclResult_t r = o.send ? ncclSend(o.buf, (size_t)o.n, ncclDouble, o.peer, ctx->comm, s)
                                    : ncclRecv(o.buf, (size_t)o.n, ncclDouble, o.peer, ctx->comm, s);
            if (r != ncclSuccess) { ncclGroupEnd(); return fail(ctx, DEFTRI_E_HIP, std::string("ncclSend/Recv: ") + ncclGetErrorString(r)); }
        }
        ncclResult_t r = ncclGroupEnd();
        if (r != ncclSuccess) return fail(ctx, DEFTRI_E_HIP, std::string("ncclGroupEnd: ") + ncclGetErrorString(r));
        return 0;
    }
    if (!ctx->xfn) return fail(ctx, DEFTRI_E_ARG, "point-sharded context without a transport");
    HIPOK(hipStreamSynchronize(s));
    for (const P2P &o : ops) {
        if ((int64_t)ctx->xstage.size() < o.n) ctx->xstage.resize((size_t)o.n);
        if (o.send) {
            HIPOK(hipMemcpy(ctx->xstage.data(), o.buf, sizeof(double) * (size_t)o.n, hipMemcpyDeviceToHost));
            if (ctx->xfn(ctx->xuser, 2, o.peer, ctx->xstage.data(), o.n) != 0) return fail(ctx, DEFTRI_E_ARG, "send callback failed");
        } else {
            if (ctx->xfn(ctx->xuser, 3, o.peer, ctx->xstage.data(), o.n) != 0) return fail(ctx, DEFTRI_E_ARG, "recv callback failed");
            HIPOK(hipMemcpy(o.buf, ctx->xstage.data(), sizeof(double) * (size_t)o.n, hipMemcpyHostToDevice));
        }
    }
    return 0;
}

// the iterative plan's transport: the context's RCCL communicator or host callback
struct CtxTransport : SpTransport {
    deftri_ctx *ctx;
    explicit CtxTransport(deftri_ctx *c) : ctx(c) {}
    int allreduce(double *dev, int64_t n, int op, hipStream_t) override { return dist_allreduce(ctx, dev, n, op); }
    int p2p(const std::vector<Op> &ops, hipStream_t st) override {
        std::vector<P2P> v;
        v.reserve(ops.size());
        for (const Op &o : ops) v.push_back({o.peer, o.send, o.buf, o.n});
        return dist_p2p(ctx, v, st);
    }
};

// plan kind of the next upload (deftri_set_plan)
bool want_iterative(const deftri_ctx *ctx, const deftri_problem_desc *d) {
    if (ctx->plan_mode == DEFTRI_PLAN_ITERATIVE) return true;
    if (ctx->plan_mode == DEFTRI_PLAN_MULTIFRONTAL) return false;
    if (ctx->lin_solver != DEFTRI_SOLVER_PCG) return false;
    if (ctx->nranks > 1) return true;
    // one GPU: the iterative plan's product outruns the sliced multifrontal one from C2 up (734 vs
    // 690 LM it/s at 100k x 2 views) and needs no analysis; small problems keep the
    // factorization (their weakly damped steps take thousands of CG iterations)
    const int64_t ndof = 6LL * d->n_pairs + d->n_scales + 3LL * d->n_points;
    return ndof >= kIterativeMinUnknowns;
}

// LevelHook of the factor / solve launchers: the DistPlan transfers whose parent front sits at
// `level` — packed contribution blocks up (factor), forward-update vectors up (forward), boundary
// solutions down (after the parent's backward level)
void dist_hook(void *user, int phase, int level) {
    deftri_ctx *ctx = (deftri_ctx *)user;
    if (ctx->hook_rc) return;
    const Symbolic &S = ctx->S;
    const DistPlan &D = S.dist;
    const DevPlan &L = ctx->L;
    std::vector<P2P> ops;
    std::vector<const DistPlan::Xfer *> mine;
    for (const auto &x : D.xfers)
        if (x.level == level && (x.src == D.rank || x.dst == D.rank)) mine.push_back(&x);
    if (mine.empty()) return;
    int rc = 0;
    if (phase == kHookFactor) {
        for (const auto *x : mine) {
            const Front &C = S.fronts[x->child];
            const int64_t n = (int64_t)x->u * (x->u + 1) / 2;
            if (x->src == D.rank) launch_pack_cb(L, C.arena_off, C.m, C.s, ctx->d_xbuf + x->buf_off, ctx->st);
            ops.push_back({x->src == D.rank ? x->dst : x->src, x->src == D.rank, ctx->d_xbuf + x->buf_off, n});
        }
        rc = dist_p2p(ctx, ops);
        if (!rc)
            for (const auto *x : mine)
                if (x->dst == D.rank) launch_ea_packed(L, x->ea_off, x->nea, ctx->d_xbuf + x->buf_off, ctx->st);
    } else if (phase == kHookForward) {
        for (const auto *x : mine) {
            const Front &C = S.fronts[x->child];
            ops.push_back({x->src == D.rank ? x->dst : x->src, x->src == D.rank, L.vec + C.vec_off + C.s, (int64_t)x->u});
        }
        rc = dist_p2p(ctx, ops);
    } else {
        for (const auto *x : mine) {
            const Front &C = S.fronts[x->child];
            const int32_t *idx = L.fd.rows + C.rows_off + C.s;
            if (x->dst == D.rank) launch_gather_idx(x->u, idx, ctx->hook_x, ctx->d_xbuf + x->buf_off, ctx->st);
            ops.push_back({x->dst == D.rank ? x->src : x->dst, x->dst == D.rank, ctx->d_xbuf + x->buf_off, (int64_t)x->u});
        }
        rc = dist_p2p(ctx, ops);
        if (!rc)
            for (const auto *x : mine) {
                const Front &C = S.fronts[x->child];
                if (x->src == D.rank)
                    launch_scatter_idx(x->u, L.fd.rows + C.rows_off + C.s, ctx->d_xbuf + x->buf_off, ctx->hook_x, ctx->st);
            }
    }
    if (rc) ctx->hook_rc = rc;
}

// the rank's problem: the whole state, the edges it owns (DistPlan::own_*)
void subset_edges(const HostProblem &full, const DistPlan &D, HostProblem &h) {
    h = HostProblem();
    h.points = full.points; h.tg = full.tg; h.scales = full.scales; h.cam_pose = full.cam_pose;
    h.cam_kb8 = full.cam_kb8; h.rot = full.rot; h.pair_area = full.pair_area; h.pair_info = full.pair_info;
    for (int32_t e : D.own_rep) {
        h.rep_point.push_back(full.rep_point[e]); h.rep_cam.push_back(full.rep_cam[e]);
        h.rep_obs.push_back(full.rep_obs[2 * (size_t)e]); h.rep_obs.push_back(full.rep_obs[2 * (size_t)e + 1]);
        h.rep_info.push_back(full.rep_info[e]);
    }
    for (int32_t e : D.own_dep) {
        h.dep_point.push_back(full.dep_point[e]); h.dep_scale.push_back(full.dep_scale[e]);
        h.dep_cam.push_back(full.dep_cam[e]); h.dep_meas.push_back(full.dep_meas[e]);
        h.dep_info.push_back(full.dep_info[e]);
    }
    for (int32_t e : D.own_arap) {
        for (int k = 0; k < 4; k++) h.arap_pts.push_back(full.arap_pts[4 * (size_t)e + k]);
        h.arap_pair.push_back(full.arap_pair[e]);
        h.arap_rot.push_back(full.arap_rot[2 * (size_t)e]); h.arap_rot.push_back(full.arap_rot[2 * (size_t)e + 1]);
        h.arap_w.push_back(full.arap_w[e]);
    }
    h.d = full.d;
    h.d.n_rep = (int32_t)D.own_rep.size(); h.d.n_depth = (int32_t)D.own_dep.size(); h.d.n_arap = (int32_t)D.own_arap.size();
    h.d.points = h.points.data(); h.d.tg = h.tg.data(); h.d.scales = h.scales.data();
    h.d.cam_kb8 = h.cam_kb8.data(); h.d.cam_pose = h.cam_pose.data();
    h.d.rep_point = h.rep_point.data(); h.d.rep_cam = h.rep_cam.data(); h.d.rep_obs = h.rep_obs.data();
    h.d.rep_info = h.rep_info.data();
    h.d.dep_point = h.dep_point.data(); h.d.dep_scale = h.dep_scale.data(); h.d.dep_cam = h.dep_cam.data();
    h.d.dep_meas = h.dep_meas.data(); h.d.dep_info = h.dep_info.data();
    h.d.arap_pts = h.arap_pts.data(); h.d.arap_pair = h.arap_pair.data(); h.d.arap_rot = h.arap_rot.data();
    h.d.arap_w = h.arap_w.data(); h.d.rot = h.rot.data(); h.d.pair_area = h.pair_area.data();
    h.d.pair_info = h.pair_info.data();
    h.d.order_xy = nullptr;
}

// a context on the iterative plan asked for what only the multifrontal plan has (the LDL^T, the
// assembled H): analyse and upload it now from the uploaded problem, continuing from the iterative
// plan's current state (deftri_reset_state still returns to the uploaded values)
int ensure_multifrontal(deftri_ctx *ctx) {
    if (!ctx->sp_on) return 0;
    const deftri_problem_desc &d = ctx->hp.d;
    std::vector<double> pts(3 * (size_t)d.n_points), sc(d.n_scales), tg(7 * (size_t)d.n_pairs);
    int rc = ctx->sp->download(pts.data(), sc.data(), tg.data());
    if (rc) return fail(ctx, rc, ctx->sp->err);
    free_device(ctx);
    if (!analyse(ctx->hp.d, ctx->S, 32, ctx->rank, ctx->nranks)) return fail(ctx, DEFTRI_E_ARG, "analysis failed: " + ctx->S.error);
    ctx->analysed = true;
    if (ctx->dist()) subset_edges(ctx->hp, ctx->S.dist, ctx->hloc);
    rc = upload_device(ctx, ctx->dist() ? ctx->hloc : ctx->hp);
    if (rc) { free_device(ctx); return rc; }
    ctx->plan_hash = structure_hash(ctx->hp.d);
    ctx->have = true;
    DevProblem &P = ctx->P;
    HIPOK(hipMemcpy(P.points, pts.data(), sizeof(double) * pts.size(), hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(P.scales, sc.data(), sizeof(double) * sc.size(), hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(P.tg, tg.data(), sizeof(double) * tg.size(), hipMemcpyHostToDevice));
    return 0;
}

// chi2 at the current state (computeActiveErrors + activeRobustChi2) into d_scal[slot]; point-sharded:
// this rank's edges, summed over the ranks unless `reduce` is false (the caller reduces it together
// with other scalars)
// extra: one more fixed-order sum to run in the same two launches (the trial's rho denominator)
int eval_chi2_dev(deftri_ctx *ctx, bool want_jac, bool analytic, int slot, bool reduce = true,
                  const SumJob *extra = nullptr) {
    DevProblem &P = ctx->P;
    launch_linearize(P, ctx->st, want_jac, analytic);
    // sum of the three chi arrays, in edge order rep, depth, arap (three partial sums, then add)
    SumJobs J;
    J.j[0].n = P.R; J.j[0].a = P.chi_rep; J.j[0].out = ctx->d_scal + 4;
    J.j[1].n = P.D; J.j[1].a = P.chi_dep; J.j[1].out = ctx->d_scal + 5;
    J.j[2].n = P.E; J.j[2].a = P.chi_arap; J.j[2].out = ctx->d_scal + 6;
    J.nj = 3;
    if (extra) J.j[J.nj++] = *extra;
    J.total = ctx->d_scal + slot;
    launch_sum_multi(J, ctx->d_part, kRedParts, ctx->st);
    return reduce ? dist_allreduce(ctx, ctx->d_scal + slot, 1, 0) : 0;
}

double read_scal(deftri_ctx *ctx, int slot) {
    hipMemcpyAsync(ctx->hpin, ctx->d_scal + slot, sizeof(double), hipMemcpyDeviceToHost, ctx->st);
    hipStreamSynchronize(ctx->st);
    return ctx->hpin[0];
}

void push_state(deftri_ctx *ctx) {
    DevProblem &P = ctx->P;
    hipMemcpyAsync(P.points_bak, P.points, sizeof(double) * 3 * (size_t)P.P, hipMemcpyDeviceToDevice, ctx->st);
    hipMemcpyAsync(P.scales_bak, P.scales, sizeof(double) * (size_t)P.S, hipMemcpyDeviceToDevice, ctx->st);
    hipMemcpyAsync(P.tg_bak, P.tg, sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToDevice, ctx->st);
}

void pop_state(deftri_ctx *ctx) {
    DevProblem &P = ctx->P;
    hipMemcpyAsync(P.points, P.points_bak, sizeof(double) * 3 * (size_t)P.P, hipMemcpyDeviceToDevice, ctx->st);
    hipMemcpyAsync(P.scales, P.scales_bak, sizeof(double) * (size_t)P.S, hipMemcpyDeviceToDevice, ctx->st);
    hipMemcpyAsync(P.tg, P.tg_bak, sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToDevice, ctx->st);
}

// DEFTRI_TRIAL_EVENTS=1: per-trial timing events on the sequential trial path, for the factor /
// solve / update split of the report (off by default: each event record is a barrier packet, ~6 us
// of stream time per event, 4 per trial; measured 0.874 -> 0.849 ms per C2 PCG trial without them)
bool trial_events_on() {
    static const bool on = [] { const char *e = std::getenv("DEFTRI_TRIAL_EVENTS"); return e && std::atoi(e) != 0; }();
    return on;
}

void trial_ev(deftri_ctx *ctx, hipEvent_t ev, hipStream_t st) {
    if (trial_events_on()) hipEventRecord(ev, st);
}

bool use_pcg(const deftri_ctx *ctx) { return ctx->lin_solver == DEFTRI_SOLVER_PCG && ctx->pcg_avail; }

// buildSystem after a linearization.  A matrix-free PCG step reads only b and the diagonal blocks
// (k_mf_lin; with want_dvec also the diagonal per dof for max diag); every other step solver
// assembles H and b.  ensure_assembled: H for a step that falls back to the LDL^T.
void build_system(deftri_ctx *ctx, bool pcg_step, bool want_dvec = false) {
    ctx->pcg_packed = false;
    if (pcg_step && ctx->G.mf) {
        launch_mf_lin(ctx->G, want_dvec, ctx->st);
        ctx->assembled = false;
    } else {
        launch_assemble(ctx->P, ctx->L, ctx->st);
        ctx->assembled = true;
    }
}
void ensure_assembled(deftri_ctx *ctx) {
    if (ctx->assembled) return;
    launch_assemble(ctx->P, ctx->L, ctx->st);
    ctx->assembled = true;
}

int lane_count(const deftri_ctx *ctx) {
    if (ctx->dist()) return 1;              // point-sharded: one trial at a time (the transfers are per trial)
    if (use_pcg(ctx)) return 1;             // PCG steps: sequential trials (the lanes batch factorizations)
    int n = ctx->max_lanes;
    if (n <= 0) {
        n = ctx->S.factor_flops < kLaneFlopLimit ? 2 : 1;
        if (const char *e = std::getenv("DEFTRI_LM_LANES")) n = std::atoi(e);
    }
    return std::max(1, std::min(kMaxLanes, n));
}

// allocate lanes up to `want` (fewer if they would not fit in half of the free HBM); returns the
// number available (>= 1), or < 0 on an allocation error
int ensure_lanes(deftri_ctx *ctx, int want) {
    if ((int)ctx->lanes.size() >= want) return want;
    const DevProblem &P0 = ctx->P;
    const DevPlan &L0 = ctx->L;
    const int64_t plan_doubles = L0.arena_size + L0.inv_size + 2 * L0.vec_size + L0.ndof;
    const int64_t lane_doubles = 3 * (int64_t)P0.P + P0.S + 7 * (int64_t)P0.Q + P0.R + P0.D + P0.E + kRedParts + 8;
    size_t free_b = 0, total_b = 0;
    hipMemGetInfo(&free_b, &total_b);
    // the batched buffers are re-allocated for the new lane count (the old ones stay until the
    // problem is freed: lanes only grow)
    int n = want;
    while (n > 1 && 8.0 * (double)n * (double)(plan_doubles + lane_doubles) > 0.5 * (double)free_b) n--;
    if (n <= (int)ctx->lanes.size()) return std::max(1, (int)ctx->lanes.size());
    DevPlan LB = L0;
    LB.nlanes = n;
    LB.lo = LaneOff{};
    LB.lo.arena = L0.arena_size; LB.lo.inv = L0.inv_size; LB.lo.vec = L0.vec_size; LB.lo.x = L0.ndof;
    LB.lo.pflag = std::max<int64_t>(L0.npanels, 1);
    if (dalloc(ctx, &LB.arena, n * L0.arena_size) || dalloc(ctx, &LB.inv, n * std::max<int64_t>(L0.inv_size, 1)) ||
        dalloc(ctx, &LB.vec, n * L0.vec_size) || dalloc(ctx, &LB.yvec, n * L0.vec_size) ||
        dalloc(ctx, &LB.flag, n) || dalloc(ctx, &LB.pflag, n * LB.lo.pflag) || (ctx->S.trsm_fused && dalloc(ctx, &LB.wbuf, 4096 * n * LB.lo.pflag)) ||
        dalloc(ctx, &ctx->dx_lanes, n * L0.ndof))
        return -1;
    if (hipMemset(LB.pflag, 0, sizeof(int) * (size_t)(n * LB.lo.pflag)) != hipSuccess) return -1;
    ctx->LB = LB;
    while ((int)ctx->lanes.size() < n) {
        Lane ln;
        ln.P = P0;
        ln.P.points_bak = ln.P.scales_bak = ln.P.tg_bak = nullptr;
        if (dalloc(ctx, &ln.P.points, 3 * (int64_t)P0.P) || dalloc(ctx, &ln.P.scales, P0.S) ||
            dalloc(ctx, &ln.P.tg, 7 * (int64_t)P0.Q) || dalloc(ctx, &ln.P.chi_rep, P0.R) ||
            dalloc(ctx, &ln.P.chi_dep, P0.D) || dalloc(ctx, &ln.P.chi_arap, P0.E) ||
            dalloc(ctx, &ln.part, kRedParts) || dalloc(ctx, &ln.scal, 8))
            return -1;
        ctx->lanes.push_back(ln);
    }
    return n;
}

// one speculative round of nl trials with lambdas lam[0..nl): setLambda + factor + solve batched
// over the lanes, then per lane the update on a scratch copy of the state (skipped on a zero
// pivot), computeActiveErrors + activeRobustChi2 there and the rho denominator; the scalars land
// in the pinned slots (read after the caller's synchronize)
void lanes_round(deftri_ctx *ctx, int nl, const double *lam, bool analytic) {
    hipStream_t st = ctx->st;
    const DevProblem &P = ctx->P;
    DevPlan LB = ctx->LB;
    LB.nlanes = nl;
    for (int t = 0; t < nl; t++) LB.lo.lam[t] = lam[t];
    hipMemsetAsync(LB.flag, 0, sizeof(int) * nl, st);
    launch_scatter_lanes(LB, st);
    launch_factor(LB, st, st, ctx->sync_ev, 64);
    launch_solve(LB, ctx->L.b, ctx->dx_lanes, st);
    for (int t = 0; t < nl; t++) {
        Lane &ln = ctx->lanes[t];
        const double *dx = ctx->dx_lanes + (int64_t)t * ctx->L.ndof;
        hipMemcpyAsync(ln.P.points, P.points, sizeof(double) * 3 * (size_t)P.P, hipMemcpyDeviceToDevice, st);
        hipMemcpyAsync(ln.P.scales, P.scales, sizeof(double) * (size_t)P.S, hipMemcpyDeviceToDevice, st);
        hipMemcpyAsync(ln.P.tg, P.tg, sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToDevice, st);
        launch_update_state(ln.P, dx, st, LB.flag + t);
        launch_linearize(ln.P, st, false, analytic);
        launch_sum(P.R, ln.P.chi_rep, nullptr, 0, 0, ln.part, kRedParts, ln.scal + 4, st);
        launch_sum(P.D, ln.P.chi_dep, nullptr, 0, 0, ln.part, kRedParts, ln.scal + 5, st);
        launch_sum(P.E, ln.P.chi_arap, nullptr, 0, 0, ln.part, kRedParts, ln.scal + 6, st);
        launch_sum(3, ln.scal + 4, nullptr, 0, 0, ln.part, 1, ln.scal, st);
        launch_sum(ctx->S.ndof, dx, ctx->L.b, lam[t], 1, ln.part, kRedParts, ln.scal + 1, st);
        hipMemcpyAsync(ctx->lane_pin + 2 * t, ln.scal, sizeof(double) * 2, hipMemcpyDeviceToHost, st);
    }
    hipMemcpyAsync(ctx->lane_ipin, LB.flag, sizeof(int) * nl, hipMemcpyDeviceToHost, st);
}

// the accepted lane's state becomes the optimizer's state
void adopt_lane_state(deftri_ctx *ctx, int t) {
    DevProblem &P = ctx->P;
    const Lane &ln = ctx->lanes[t];
    hipMemcpyAsync(P.points, ln.P.points, sizeof(double) * 3 * (size_t)P.P, hipMemcpyDeviceToDevice, ctx->st);
    hipMemcpyAsync(P.scales, ln.P.scales, sizeof(double) * (size_t)P.S, hipMemcpyDeviceToDevice, ctx->st);
    hipMemcpyAsync(P.tg, ln.P.tg, sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToDevice, ctx->st);
}

float ev_ms(deftri_ctx *ctx, int a, int b) {
    float ms = 0;
    hipEventElapsedTime(&ms, ctx->ev[a], ctx->ev[b]);
    return ms;
}

}  // namespace

// ==========================================================================================
// C-ABI
// ==========================================================================================
using LiveCtx = deftri::LiveContexts<deftri_ctx, deftri_ctx_destroy>;

extern "C" {

int deftri_abi_version(void) { return DEFTRI_ABI_VERSION; }

int deftri_ctx_create(int32_t device, deftri_ctx **out) {
    if (!out) return DEFTRI_E_ARG;
    *out = nullptr;
    if (device < 0) {                    // host-only context
        deftri_ctx *ctx = new deftri_ctx();
        ctx->device = -1;
        *out = ctx;
        return 0;
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return DEFTRI_E_NODEVICE;
    if (device < 0 || device >= n) return DEFTRI_E_NODEVICE;
    deftri_ctx *ctx = new deftri_ctx();
    ctx->device = device;
    // the main stream (panel chain: the critical path) gets the higher priority; the side stream's
    // big trailing updates fill the CUs it leaves free
    int prio_lo = 0, prio_hi = 0;
    if (hipSetDevice(device) == hipSuccess) hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithPriority(&ctx->st, hipStreamNonBlocking, prio_hi) != hipSuccess) {
        delete ctx;
        return DEFTRI_E_HIP;
    }
    for (auto &e : ctx->ev) hipEventCreate(&e);
    if (hipHostMalloc((void **)&ctx->hpin, 32 * sizeof(double), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&ctx->ipin, 16 * sizeof(int), hipHostMallocDefault) != hipSuccess) {
        delete ctx;
        return DEFTRI_E_HIP;
    }
    for (int i = 0; i < 32; i++) ctx->hpin[i] = 0.0;
    hipStreamCreateWithPriority(&ctx->side, hipStreamNonBlocking, prio_lo);
    for (auto &e : ctx->sync_ev) hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (hipHostMalloc((void **)&ctx->lane_pin, 2 * kMaxLanes * sizeof(double), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&ctx->lane_ipin, kMaxLanes * sizeof(int), hipHostMallocDefault) != hipSuccess) {
        deftri_ctx_destroy(ctx);
        return DEFTRI_E_HIP;
    }
    LiveCtx::add(ctx);
    *out = ctx;
    return 0;
}

int deftri_ctx_destroy(deftri_ctx *ctx) {
    if (!ctx) return 0;
    if (ctx->device < 0) { delete ctx; return 0; }
    LiveCtx::remove(ctx);
    hipSetDevice(ctx->device);
    free_device(ctx);
    ctx->gdev.reset();
    delete ctx->sp_tr;
    ctx->sp_tr = nullptr;
    if (ctx->comm) ncclCommDestroy(ctx->comm);
    for (auto &e : ctx->ev) if (e) hipEventDestroy(e);
    for (auto &e : ctx->sync_ev) if (e) hipEventDestroy(e);
    if (ctx->lane_pin) hipHostFree(ctx->lane_pin);
    if (ctx->lane_ipin) hipHostFree(ctx->lane_ipin);
    if (ctx->side) hipStreamDestroy(ctx->side);
    if (ctx->st) hipStreamDestroy(ctx->st);
    if (ctx->hpin) hipHostFree(ctx->hpin);
    if (ctx->ipin) hipHostFree(ctx->ipin);
    delete ctx;
    return 0;
}

const char *deftri_last_error(const deftri_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int deftri_set_jacobian_mode(deftri_ctx *ctx, int32_t analytic) {
    if (!ctx || analytic < 0 || analytic > 1) return DEFTRI_E_ARG;
    ctx->analytic_jac = analytic;
    return 0;
}

int deftri_set_factor_precision(deftri_ctx *ctx, int32_t fp32_updates) {
    if (!ctx || fp32_updates < 0 || fp32_updates > 1) return DEFTRI_E_ARG;
    ctx->f32_update = fp32_updates;
    ctx->L.f32_update = fp32_updates;
    ctx->LB.f32_update = fp32_updates;
    drop_trial_graph(ctx);                 // the captured trial holds the previous kernel choice
    return 0;
}

int deftri_set_linear_solver(deftri_ctx *ctx, int32_t solver, double tol, int32_t max_iterations) {
    if (!ctx || (solver != DEFTRI_SOLVER_DIRECT && solver != DEFTRI_SOLVER_PCG) || !(tol < 1.0) ||
        max_iterations > kPcgMaxIt)
        return DEFTRI_E_ARG;
    ctx->lin_solver = solver;
    ctx->pcg_tol = tol > 0 ? tol : kPcgDefaultTol;
    ctx->pcg_max_it = max_iterations > 0 ? max_iterations : 0;   // 0: the plan's cost-model budget
    if (ctx->sp) { ctx->sp->tol = ctx->pcg_tol; ctx->sp->max_it = ctx->pcg_max_it; }
    return 0;
}

int deftri_last_step_info(const deftri_ctx *ctx, int32_t *pcg_iterations, int32_t *pcg_converged) {
    if (!ctx || !pcg_iterations || !pcg_converged) return DEFTRI_E_ARG;
    if (ctx->sp_on) {
        *pcg_iterations = ctx->sp->step_its;
        *pcg_converged = ctx->sp->step_solved;
        return 0;
    }
    *pcg_iterations = ctx->pcg_step_its;
    *pcg_converged = ctx->pcg_step_solved;
    return 0;
}

int deftri_debug_sp_product(deftri_ctx *ctx, const deftri_problem_desc *desc, const double *jarap, const double *warap,
                            const double *jrep, const double *wrep, const double *jdep, const double *wdep,
                            double lambda, const double *p, double *q, int64_t n, int64_t *stats) {
    if (!ctx || !desc || !p || !q) return DEFTRI_E_ARG;
    int rc = validate(ctx, desc);
    if (rc) return rc;
    if ((desc->n_arap && (!jarap || !warap)) || (desc->n_rep && (!jrep || !wrep)) || (desc->n_depth && (!jdep || !wdep)))
        return fail(ctx, DEFTRI_E_ARG, "missing Jacobian / weight arrays");
    if (n != 6LL * desc->n_pairs + desc->n_scales + 3LL * desc->n_points) return fail(ctx, DEFTRI_E_ARG, "size mismatch");
    if (ctx->nranks > 1 && !ctx->xfn) return fail(ctx, DEFTRI_E_ARG, "the emulation needs the callback transport");
    SpPlanHost H;
    std::string err;
    // DEFTRI_SP_EMULATE_TILE=1 (read per call): one pair — the tile layout's product instead (sharded:
    // this rank's rows and its share of the heavy sums, all-reduced through the transport)
    const bool tile = std::getenv("DEFTRI_SP_EMULATE_TILE") != nullptr;
    if (!build_sp_plan(*desc, ctx->rank, ctx->nranks, false, H, err, tile)) return fail(ctx, DEFTRI_E_ARG, err);
    if (tile) {
        if (!H.tile) return fail(ctx, DEFTRI_E_ARG, "no tile layout: " + H.tile_why);
        rc = sp_emulate_tile_product(*desc, H, jarap, warap, jrep, wrep, jdep, wdep, lambda, p, q, err);
        if (rc) return fail(ctx, DEFTRI_E_ARG, "tile layout: " + err);
        if (ctx->nranks > 1) {
            if (ctx->xfn(ctx->xuser, 0, -1, q, H.hd) != 0) return fail(ctx, DEFTRI_E_ARG, "all-reduce callback failed");
            for (int64_t k = 0; k < H.hd; k++) q[k] += lambda * p[k];
        }
    } else {
        std::function<int(int, int, double *, int64_t)> xf = [ctx](int op, int peer, double *buf, int64_t cnt) {
            return ctx->xfn(ctx->xuser, op, peer, buf, cnt);
        };
        rc = sp_emulate_product(*desc, H, jarap, warap, jrep, wrep, jdep, wdep, lambda, p, q, xf);
        if (rc) return fail(ctx, DEFTRI_E_ARG, "transfer callback failed");
    }
    if (stats) {
        stats[0] = H.hi - H.lo;
        stats[1] = tile ? 0 : H.halo_rows;
        stats[2] = (int64_t)H.arap_ids.size();
        stats[3] = H.n_arap_owned;
    }
    return 0;
}

int deftri_set_pair_window(deftri_ctx *ctx, int32_t window) {
    if (!ctx || window < 0) return DEFTRI_E_ARG;
    ctx->pair_window = window;
    return 0;
}

int deftri_set_plan(deftri_ctx *ctx, int32_t plan) {
    if (!ctx || plan < DEFTRI_PLAN_AUTO || plan > DEFTRI_PLAN_ITERATIVE) return DEFTRI_E_ARG;
    ctx->plan_mode = plan;
    return 0;
}

int deftri_set_jacobian_storage(deftri_ctx *ctx, int32_t fp32) {
    if (!ctx || fp32 < 0 || fp32 > 1) return DEFTRI_E_ARG;
    ctx->jac_fp32 = fp32;
    return 0;
}

int deftri_get_plan_info(const deftri_ctx *ctx, deftri_plan_info *info) {
    if (!ctx || !info) return DEFTRI_E_ARG;
    std::memset(info, 0, sizeof(*info));
    info->rank = ctx->rank;
    info->nranks = ctx->nranks;
    if (ctx->sp_on) {
        const SpSolver &s = *ctx->sp;
        info->plan = DEFTRI_PLAN_ITERATIVE;
        info->own_rows = s.own_rows();
        info->halo_rows = s.halo_rows();
        info->local_arap_edges = s.n_arap_local();
        info->n_unknowns = s.ndof();
        info->phase1_blocks = s.n_blocks();
        info->row_blocks = s.n_row_blocks();
        info->product_bytes = s.product_bytes();
        info->jacobian_fp32 = s.fp32_jac;
        info->cg_launches = s.cg_launches();
        info->cg_collectives = s.cg_collectives();
        info->sharded = s.sharded() ? 1 : 0;
        info->survey_bytes = s.survey_bytes();
        info->tiles = s.n_tiles();
        info->halo_overlap = s.halo_overlap() ? 1 : 0;
        return 0;
    }
    if (!ctx->have) return DEFTRI_E_NOPROBLEM;
    info->plan = DEFTRI_PLAN_MULTIFRONTAL;
    info->n_unknowns = ctx->S.ndof;
    info->product_bytes = ctx->pcg_bytes;
    return 0;
}

int deftri_set_lm_lanes(deftri_ctx *ctx, int32_t lanes) {
    if (!ctx || lanes < 0 || lanes > kMaxLanes) return DEFTRI_E_ARG;
    ctx->max_lanes = lanes;
    return 0;
}

int deftri_dist_init_rccl(deftri_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t id[128]) {
    if (!ctx || nranks < 1 || rank < 0 || rank >= nranks || !id) return DEFTRI_E_ARG;
    if (ctx->device < 0) return fail(ctx, DEFTRI_E_NODEVICE, "host-only context");
    hipSetDevice(ctx->device);
    free_device(ctx);
    ctx->analysed = false;
    if (ctx->comm) { ncclCommDestroy(ctx->comm); ctx->comm = nullptr; }
    ctx->xfn = nullptr; ctx->xuser = nullptr;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclResult_t r = ncclCommInitRank(&ctx->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        ctx->comm = nullptr;
        return fail(ctx, DEFTRI_E_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    ctx->rank = rank; ctx->nranks = nranks;
    return 0;
}

int deftri_dist_set_transport(deftri_ctx *ctx, int32_t nranks, int32_t rank, deftri_xfer_fn fn, void *user) {
    if (!ctx || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !fn)) return DEFTRI_E_ARG;
    if (ctx->device >= 0) { hipSetDevice(ctx->device); free_device(ctx); }
    ctx->analysed = false;
    if (ctx->comm) { ncclCommDestroy(ctx->comm); ctx->comm = nullptr; }
    ctx->xfn = fn; ctx->xuser = user;
    ctx->rank = rank; ctx->nranks = nranks;
    return 0;
}

int deftri_plan_vertex_order(const deftri_ctx *ctx, int64_t *order, int64_t nv) {
    if (!ctx || !order) return DEFTRI_E_ARG;
    if (!ctx->analysed) return DEFTRI_E_NOPROBLEM;
    if (nv != ctx->S.nv) return DEFTRI_E_ARG;
    for (int64_t v = 0; v < nv; v++) order[ctx->S.elim_pos[v]] = v;
    return 0;
}

int deftri_dist_vertex_owner(const deftri_ctx *ctx, int32_t *owner, int64_t nv) {
    if (!ctx || !owner) return DEFTRI_E_ARG;
    if (ctx->sp_on) return ctx->sp->vertex_owner(owner, nv);
    if (!ctx->analysed) return DEFTRI_E_NOPROBLEM;
    if (nv != ctx->S.nv) return DEFTRI_E_ARG;
    std::memcpy(owner, ctx->S.dist.vertex_owner.data(), sizeof(int32_t) * (size_t)nv);
    return 0;
}

int deftri_dist_owned_edges(const deftri_ctx *ctx, uint8_t *rep, uint8_t *dep, uint8_t *arap) {
    if (!ctx) return DEFTRI_E_ARG;
    if (!ctx->analysed) return DEFTRI_E_NOPROBLEM;
    const DistPlan &D = ctx->S.dist;
    const deftri_problem_desc &d = ctx->hp.d;
    if (rep) { std::memset(rep, 0, (size_t)d.n_rep); for (int32_t e : D.own_rep) rep[e] = 1; }
    if (dep) { std::memset(dep, 0, (size_t)d.n_depth); for (int32_t e : D.own_dep) dep[e] = 1; }
    if (arap) { std::memset(arap, 0, (size_t)d.n_arap); for (int32_t e : D.own_arap) arap[e] = 1; }
    return 0;
}

int64_t deftri_num_unknowns(const deftri_ctx *ctx) {
    if (ctx && ctx->sp_on) return ctx->sp->ndof();
    return (ctx && ctx->have) ? ctx->S.ndof : -1;
}

int deftri_problem_analyse(deftri_ctx *ctx, const deftri_problem_desc *desc) {
    if (!ctx) return DEFTRI_E_ARG;
    int rc = validate(ctx, desc);
    if (rc) return rc;
    if (ctx->device >= 0) { hipSetDevice(ctx->device); free_device(ctx); }
    ctx->have = false;
    copy_host(ctx->hp, desc);
    ctx->plan_hash = 0;
    if (!analyse(ctx->hp.d, ctx->S, 32, ctx->rank, ctx->nranks)) return fail(ctx, DEFTRI_E_ARG, "analysis failed: " + ctx->S.error);
    ctx->analysed = true;
    return 0;
}

int deftri_plan_stats(const deftri_ctx *ctx, deftri_report *rep) {
    if (!ctx || !rep) return DEFTRI_E_ARG;
    if (!ctx->analysed) return DEFTRI_E_NOPROBLEM;
    std::memset(rep, 0, sizeof(*rep));
    rep->n_unknowns = ctx->S.ndof;
    rep->nnz_factor = ctx->S.nnz_factor;
    rep->factor_flops = ctx->S.factor_flops;
    rep->n_fronts = (int32_t)ctx->S.fronts.size();
    rep->n_levels = ctx->S.nlevels;
    rep->rank = ctx->rank;
    rep->nranks = ctx->nranks;
    rep->factor_flops_total = ctx->S.dist.factor_flops_total;
    rep->plan_reuses = ctx->plan_reuses;
    return 0;
}

int deftri_debug_plan_solve(deftri_ctx *ctx, const double *H, double lambda, const double *rhs, double *x,
                            int64_t n) {
    if (!ctx || !H || !rhs || !x) return DEFTRI_E_ARG;
    if (!ctx->analysed) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem analysed");
    if (n != ctx->S.ndof) return fail(ctx, DEFTRI_E_ARG, "size mismatch");
    return plan_emulate_solve(ctx->S, H, lambda, rhs, x) == 0 ? 0 : fail(ctx, DEFTRI_E_NUMERIC, "zero pivot");
}

int deftri_debug_plan_solve_dist(deftri_ctx *ctx, const double *Hq, double lambda, const double *bq, double *x,
                                 int64_t n) {
    if (!ctx || !Hq || !bq || !x) return DEFTRI_E_ARG;
    if (!ctx->analysed) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem analysed");
    if (n != ctx->S.ndof) return fail(ctx, DEFTRI_E_ARG, "size mismatch");
    if (ctx->dist() && !ctx->xfn) return fail(ctx, DEFTRI_E_ARG, "the emulation needs the callback transport");
    std::function<int(int, int, double *, int64_t)> xf = [ctx](int op, int peer, double *buf, int64_t cnt) {
        return ctx->xfn(ctx->xuser, op, peer, buf, cnt);
    };
    // forward gather reads the full rhs on the rank's own rows and the partial one on the boundary
    // of its top front: both are b_q here (the test's b_q is zero outside the rank's contributions)
    const int rc = plan_emulate_solve(ctx->S, Hq, lambda, bq, x, ctx->dist() ? &xf : nullptr, ctx->dist() ? bq : nullptr);
    if (rc == -2) return fail(ctx, DEFTRI_E_ARG, "transfer callback failed");
    return rc == 0 ? 0 : fail(ctx, DEFTRI_E_NUMERIC, "zero pivot");
}

namespace {
int pcg_step(deftri_ctx *ctx, double lambda, const double *rhs, bool &solved, int &its);
}

int deftri_profile_trial(deftri_ctx *ctx, double lambda, deftri_kernel_stat *stats, int32_t max_stats,
                         int32_t *n_stats) {
    if (!ctx || !stats || !n_stats) return DEFTRI_E_ARG;
    if (!ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(ctx->device);
    HIPOK(hipStreamSynchronize(ctx->st));
    KProf prof;
    if (ctx->sp_on && ctx->lin_solver != DEFTRI_SOLVER_PCG) {
        const int rc0 = ensure_multifrontal(ctx);     // the factorization's kernels asked for
        if (rc0) return rc0;
    }
    if (ctx->sp_on) {
        int rc = ctx->sp->profile_trial(lambda, prof, ctx->prof_analytic);
        if (rc) return fail(ctx, rc, ctx->sp->err);
        const int its = ctx->sp->step_its;
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
            if (!std::strcmp(stats[k].name, "sp_phase1") || !std::strcmp(stats[k].name, "sp_tile"))
                stats[k].bytes = ctx->sp->product_bytes_phase(1) * its;
            if (!std::strcmp(stats[k].name, "sp_phase2") || !std::strcmp(stats[k].name, "sp_tupd"))
                stats[k].bytes = ctx->sp->product_bytes_phase(2) * its;
        }
        for (hipEvent_t e : prof.pool) hipEventDestroy(e);
        *n_stats = n;
        return 0;
    }
    set_profiler(&prof);
    // point-sharded: a collective (every rank profiles its part of the same trial)
    LevelHook hook = ctx->dist() ? dist_hook : nullptr;
    ctx->hook_rc = 0;
    ctx->hook_x = ctx->d_dx;
    int rc = eval_chi2_dev(ctx, true, ctx->prof_analytic, 0);
    build_system(ctx, use_pcg(ctx));
    hipMemsetAsync(ctx->L.flag, 0, sizeof(int), ctx->st);
    bool solved = false;
    int its = 0;
    if (!rc && use_pcg(ctx)) {
        // the configured PCG step: solved once to learn its iteration count, then replayed with
        // exactly that many (update, product) pairs under the profiler
        set_profiler(nullptr);
        rc = pcg_step(ctx, lambda, ctx->L.b, solved, its);
        set_profiler(&prof);
        if (!rc && solved) {
            const PcgDev &G = ctx->G;
            if (!G.mf) launch_pcg_repack(G, ctx->L.hval, ctx->st);   // once per LM iteration (after the assembly)
            launch_pcg_setup(G, ctx->L.hval, ctx->L.b, lambda, ctx->d_dx, ctx->st);
            launch_pcg_product(G, 0, ctx->L.hval, lambda, ctx->st);
            for (int j = 0; j < its; j++) {
                launch_pcg_heavy(G, j, ctx->L.hval, lambda, ctx->st);
                launch_pcg_update(G, j, lambda, ctx->d_dx, ctx->st);
                // the product after the last update only runs the convergence test: not profiled, so
                // the product's statistics cover exactly the `its` active launches
                if (j + 1 == its) set_profiler(nullptr);
                launch_pcg_product(G, j + 1, ctx->L.hval, lambda, ctx->st);
            }
            set_profiler(&prof);
        }
    }
    if (!solved) {
        ensure_assembled(ctx);
        launch_scatter(ctx->L, lambda, ctx->st);
        launch_factor(ctx->L, ctx->st, ctx->side, ctx->sync_ev, 64, hook, ctx);
        launch_solve(ctx->L, ctx->L.b, ctx->d_dx, ctx->st, ctx->dist() ? ctx->L.b : nullptr, hook, ctx);
    }
    set_profiler(nullptr);
    if (rc) return rc;
    if (ctx->hook_rc) return ctx->hook_rc;
    HIPOK(hipStreamSynchronize(ctx->st));
    int32_t n = 0;
    const bool dump = std::getenv("DEFTRI_PROFILE_DUMP") != nullptr;
    for (const auto &r : prof.recs) {
        float ms = 0;
        hipEventElapsedTime(&ms, r.e0, r.e1);
        if (dump) std::fprintf(stderr, "[prof] %s %u %.4f %.6g %d\n", r.name, r.grid, ms, r.work, r.level);
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
    const Symbolic &S = ctx->S;
    for (int32_t k = 0; k < n; k++) {
        if (!std::strcmp(stats[k].name, "update")) stats[k].flops = S.update_flops;
        if (!std::strcmp(stats[k].name, "diag")) stats[k].flops = S.diag_flops;
        if (!std::strcmp(stats[k].name, "trsm")) stats[k].flops = S.trsm_flops;
        if (!std::strcmp(stats[k].name, "lin_arap")) stats[k].bytes = (double)ctx->P.E * (16 + 8 * 12 + 8 * 18 + 3 * 8);
        // the product's compulsory traffic per active launch: entries + block values
        // in both orientations + p_prev / z of the row's own dofs + p / q written
        if (!std::strcmp(stats[k].name, "pcg_product")) stats[k].bytes = ctx->pcg_bytes * its;
        if (!std::strcmp(stats[k].name, "pcg_product")) stats[k].flops = ctx->pcg_flops * its;
    }
    for (hipEvent_t e : prof.pool) hipEventDestroy(e);
    *n_stats = n;
    return 0;
}

int64_t deftri_sizeof(int32_t which) {
    switch (which) {
        case 0: return (int64_t)sizeof(deftri_problem_desc);
        case 1: return (int64_t)sizeof(deftri_lm_params);
        case 2: return (int64_t)sizeof(deftri_report);
        case 3: return (int64_t)sizeof(deftri_keyframe);
        case 4: return (int64_t)sizeof(deftri_map);
        case 5: return (int64_t)sizeof(deftri_ba_desc);
        case 6: return (int64_t)sizeof(deftri_pixels_error);
        case 7: return (int64_t)sizeof(deftri_plan_info);
        case 8: return (int64_t)sizeof(deftri_deformation_params);
        case 9: return (int64_t)sizeof(deftri_deformation_report);
        case 10: return (int64_t)sizeof(deftri_deformation_eval);
        default: return -1;
    }
}

int deftri_problem_upload(deftri_ctx *ctx, const deftri_problem_desc *desc) {
    if (!ctx) return DEFTRI_E_ARG;
    if (ctx->device < 0) return fail(ctx, DEFTRI_E_NODEVICE, "host-only context");
    hipSetDevice(ctx->device);
    // DEFTRI_UPLOAD_TIMING=1: the call's host stages before the plan build
    static const bool utiming = std::getenv("DEFTRI_UPLOAD_TIMING") != nullptr;
    auto ut = std::chrono::steady_clock::now();
    auto ulap = [&](const char *w) {
        if (!utiming) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[deftri upload] %-22s %7.2f ms\n", w, std::chrono::duration<double, std::milli>(t - ut).count());
        ut = t;
    };
    int rc = validate(ctx, desc);
    if (rc) return rc;
    ulap("validate");
    if (want_iterative(ctx, desc)) {
        static const bool no_cache = std::getenv("DEFTRI_NO_PLAN_CACHE") != nullptr;
        if (!no_cache && ctx->sp_on && ctx->sp && ctx->sp->fp32_jac == ctx->jac_fp32 && same_structure(ctx->hp.d, *desc) &&
            same_order_coordinates(ctx->hp.d, *desc)) {
            // the plan (row order, shards, wave layout) depends only on the structure and the
            // ordering coordinates: reuse it and copy the values
            copy_host(ctx->hp, desc);
            ctx->sp->tol = ctx->pcg_tol;
            ctx->sp->max_it = ctx->pcg_max_it;
            rc = ctx->sp->refresh(*desc);
            if (rc) { ctx->err = ctx->sp->err; free_device(ctx); return rc; }
            ctx->plan_reuses++;
            return 0;
        }
        // the point-sharded iterative plan: no ordering, no symbolic analysis, no factor
        ulap("structure check");
        free_device(ctx, true);
        ulap("free device");
        ctx->plan_hash = 0;
        ctx->analysed = false;
        copy_host(ctx->hp, desc);
        ulap("copy host");
        if (!ctx->sp_tr) ctx->sp_tr = new CtxTransport(ctx);
        ctx->sp.reset(new SpSolver(ctx->device, ctx->st, ctx->rank, ctx->nranks, ctx->sp_tr, ctx->comm != nullptr));
        ulap("solver object");
        ctx->sp->tol = ctx->pcg_tol;
        ctx->sp->max_it = ctx->pcg_max_it;
        ctx->sp->fp32_jac = ctx->jac_fp32;
        ctx->sp->before_alloc = [ctx] { join_reaper(ctx); };
        rc = ctx->sp->upload(*desc);
        if (rc) { ctx->err = ctx->sp->err; ctx->sp.reset(); return rc; }
        ctx->sp_on = true;
        ctx->have = true;
        return 0;
    }
    const uint64_t hsh = structure_hash(*desc);
    static const bool no_cache = std::getenv("DEFTRI_NO_PLAN_CACHE") != nullptr;
    if (ctx->have && ctx->analysed && hsh == ctx->plan_hash && !no_cache && same_structure(ctx->hp.d, *desc)) {
        copy_host(ctx->hp, desc);
        if (ctx->dist()) subset_edges(ctx->hp, ctx->S.dist, ctx->hloc);
        rc = refresh_values(ctx, ctx->dist() ? ctx->hloc : ctx->hp);
        if (rc) { free_device(ctx); return rc; }
        ctx->plan_reuses++;
        return 0;
    }
    free_device(ctx);
    ctx->plan_hash = hsh;
    copy_host(ctx->hp, desc);
    if (!analyse(ctx->hp.d, ctx->S, 32, ctx->rank, ctx->nranks)) return fail(ctx, DEFTRI_E_ARG, "analysis failed: " + ctx->S.error);
    ctx->analysed = true;
    if (ctx->dist()) subset_edges(ctx->hp, ctx->S.dist, ctx->hloc);
    rc = upload_device(ctx, ctx->dist() ? ctx->hloc : ctx->hp);
    if (rc) { free_device(ctx); return rc; }
    ctx->have = true;
    return 0;
}

int deftri_reset_state(deftri_ctx *ctx) {
    if (!ctx || !ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    if (ctx->sp_on) { int rc = ctx->sp->reset_state(); return rc ? fail(ctx, rc, ctx->sp->err) : 0; }
    DevProblem &P = ctx->P;
    HIPOK(hipMemcpyAsync(P.points, ctx->init_state[0], sizeof(double) * 3 * (size_t)P.P, hipMemcpyDeviceToDevice, ctx->st));
    HIPOK(hipMemcpyAsync(P.scales, ctx->init_state[1], sizeof(double) * (size_t)P.S, hipMemcpyDeviceToDevice, ctx->st));
    HIPOK(hipMemcpyAsync(P.tg, ctx->init_state[2], sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToDevice, ctx->st));
    HIPOK(hipStreamSynchronize(ctx->st));
    return 0;
}

namespace {
// One LM step by PCG into ctx->d_dx, in two halves so the LM loop can enqueue the trial's update
// and chi2 behind the first one and pay a single host round trip when the prediction holds:
//   pcg_start: repack (after an assembly), setup, product(0), then n x (heavy, update, product) with
//              n = the previous converged solve's count + 1 (the product launch carries the
//              convergence test; launches past convergence return at once); no synchronization.
//   pcg_poll:  reads the record of the last product; while still running, further chunks of 4
//              iterations with a read-back each.  solved = false: budget exhausted, breakdown, or a
//              preconditioner block not positive definite — the caller factors instead.
void pcg_limits(deftri_ctx *ctx) {
    ctx->G.max_it = ctx->pcg_max_it > 0 ? ctx->pcg_max_it : ctx->pcg_auto_it;
    ctx->G.tol2 = ctx->pcg_tol * ctx->pcg_tol;
}

// rec_cleared: the trial's prologue (launch_trial_begin, after pcg_limits) cleared the records
void pcg_start(deftri_ctx *ctx, double lambda, const double *rhs, int &j, bool rec_cleared = false) {
    PcgDev &G = ctx->G;
    const DevPlan &L = ctx->L;
    pcg_limits(ctx);
    if (!ctx->pcg_packed && !G.mf) {
        launch_pcg_repack(G, L.hval, ctx->st);
        ctx->pcg_packed = true;
    }
    launch_pcg_setup(G, L.hval, rhs, lambda, ctx->d_dx, ctx->st, rec_cleared);
    launch_pcg_product(G, 0, L.hval, lambda, ctx->st);
    j = 0;
    const int n = std::min(std::max(2, ctx->pcg_last_its + 1), G.max_it);
    for (int k = 0; k < n; k++, j++) {
        launch_pcg_heavy(G, j, ctx->L.hval, lambda, ctx->st);
        launch_pcg_update(G, j, lambda, ctx->d_dx, ctx->st);
        launch_pcg_product(G, j + 1, L.hval, lambda, ctx->st);
    }
}

// the record of product j (iteration j's convergence verdict) into the pinned staging
int pcg_fetch(deftri_ctx *ctx, int j) {
    HIPOK(hipMemcpyAsync(ctx->hpin + 16, ctx->G.rec + (size_t)kPcgRec * (j + 1), sizeof(double) * kPcgRec,
                         hipMemcpyDeviceToHost, ctx->st));
    return 0;
}

// after a synchronization that covered pcg_fetch(j): 1 converged, 0 still running, -1 given up
int pcg_verdict(deftri_ctx *ctx, int j, int &its) {
    const double *rec = ctx->hpin + 16;
    const int status = (int)rec[PR_STATUS];
    if (status == kPcgConverged) {
        its = (int)rec[PR_ITS];
        ctx->pcg_last_its = its;
        ctx->pcg_step_its = its;
        ctx->pcg_step_solved = 1;
        return 1;
    }
    if (status != kPcgRunning || j >= ctx->G.max_it) {
        its = j;
        ctx->pcg_step_its = its;
        ctx->pcg_step_solved = 0;
        return -1;
    }
    return 0;
}

int pcg_poll(deftri_ctx *ctx, double lambda, int &j, bool &solved, int &its) {
    PcgDev &G = ctx->G;
    for (;;) {
        int rc = pcg_fetch(ctx, j);
        if (rc) return rc;
        HIPOK(hipStreamSynchronize(ctx->st));
        const int v = pcg_verdict(ctx, j, its);
        if (v != 0) { solved = v > 0; return 0; }
        const int n = std::min(4, G.max_it - j);
        for (int k = 0; k < n; k++, j++) {
            launch_pcg_heavy(G, j, ctx->L.hval, lambda, ctx->st);
            launch_pcg_update(G, j, lambda, ctx->d_dx, ctx->st);
            launch_pcg_product(G, j + 1, ctx->L.hval, lambda, ctx->st);
        }
    }
}

int pcg_step(deftri_ctx *ctx, double lambda, const double *rhs, bool &solved, int &its) {
    int j = 0;
    solved = false;
    its = 0;
    pcg_start(ctx, lambda, rhs, j);
    return pcg_poll(ctx, lambda, j, solved, its);
}

// the sequential trial (scatter + factorization + solve) as one graph launch: single stream, no
// cross-rank hooks, no per-launch profiling, no fused-TRSM epochs
bool trial_graph_usable(const deftri_ctx *ctx) {
    if (ctx->trial_graph_failed || ctx->dist() || ctx->S.trsm_fused || profiling()) return false;
    for (const auto &lv : ctx->L.levels)
        for (const auto &stp : lv.steps)
            if (stp.stream != 0) return false;
    return true;
}

// enqueue one trial's scatter + factor + solve at lambda (already in ctx->d_lam on the stream's
// timeline); returns false when the caller must launch the kernels itself
bool launch_trial_graph(deftri_ctx *ctx) {
    if (!trial_graph_usable(ctx)) return false;
    if (!ctx->trial_graph) {
        hipGraph_t g = nullptr;
        if (hipStreamBeginCapture(ctx->st, hipStreamCaptureModeThreadLocal) != hipSuccess) {
            if (std::getenv("DEFTRI_GRAPH_LOG")) std::fprintf(stderr, "[deftri] trial graph: capture refused\n");
            ctx->trial_graph_failed = true;
            return false;
        }
        launch_scatter(ctx->L, 0.0, ctx->st, ctx->d_lam);
        launch_factor(ctx->L, ctx->st, ctx->side, ctx->sync_ev, 64);
        launch_solve(ctx->L, ctx->L.b, ctx->d_dx, ctx->st);
        hipGraphExec_t ex = nullptr;
        if (hipStreamEndCapture(ctx->st, &g) != hipSuccess || !g ||
            hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) != hipSuccess) {
            if (g) hipGraphDestroy(g);
            (void)hipGetLastError();
            if (std::getenv("DEFTRI_GRAPH_LOG")) std::fprintf(stderr, "[deftri] trial graph: capture failed\n");
            ctx->trial_graph_failed = true;
            return false;
        }
        hipGraphDestroy(g);
        ctx->trial_graph = ex;
        if (std::getenv("DEFTRI_GRAPH_LOG")) std::fprintf(stderr, "[deftri] trial graph captured\n");
    }
    return hipGraphLaunch(ctx->trial_graph, ctx->st) == hipSuccess;
}
}  // namespace

int deftri_solve_lm(deftri_ctx *ctx, const deftri_lm_params *prm, deftri_report *rep) {
    if (!ctx || !prm) return DEFTRI_E_ARG;
    if (!ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(ctx->device);
    deftri_report local{};
    deftri_report &R = rep ? *rep : local;
    std::memset(&R, 0, sizeof(R));
    if (ctx->sp_on && ctx->lin_solver != DEFTRI_SOLVER_PCG) {
        const int rc0 = ensure_multifrontal(ctx);     // LDL^T steps asked for: the multifrontal plan
        if (rc0) return rc0;
    }
    if (ctx->sp_on) {
        ctx->prof_analytic = prm->analytic_jacobians != 0;
        int rc = ctx->sp->solve_lm(*prm, R);
        R.plan_reuses = ctx->plan_reuses;
        return rc ? fail(ctx, rc, ctx->sp->err) : 0;
    }
    R.n_unknowns = ctx->S.ndof;
    R.nnz_factor = ctx->S.nnz_factor;
    R.factor_flops = ctx->S.factor_flops;
    R.n_fronts = (int32_t)ctx->S.fronts.size();
    R.n_levels = ctx->S.nlevels;
    R.rank = ctx->rank;
    R.nranks = ctx->nranks;
    R.factor_flops_total = ctx->S.dist.factor_flops_total;
    R.plan_reuses = ctx->plan_reuses;
    const int max_trials = prm->max_trials > 0 ? prm->max_trials : 10;
    const double tau = prm->tau > 0 ? prm->tau : 1e-5;
    const bool analytic = prm->analytic_jacobians != 0;
    ctx->prof_analytic = analytic;
    const bool dist = ctx->dist();
    ctx->hook_rc = 0;
    LevelHook hook = dist ? dist_hook : nullptr;
    int rc = 0;
    DevProblem &P = ctx->P;
    DevPlan &L = ctx->L;
    auto t_start = std::chrono::steady_clock::now();
    double lambda = 0, ni = 2;
    double t_lin = 0, t_fac = 0, t_sol = 0, t_upd = 0;
    int status = DEFTRI_STATUS_OK, it;
    if ((rc = eval_chi2_dev(ctx, false, analytic, 0))) return rc;
    R.chi2_initial = read_scal(ctx, 0);
    double currentChi = R.chi2_initial;
    int nlanes = std::min(lane_count(ctx), max_trials);
    if (nlanes > 1) {
        nlanes = ensure_lanes(ctx, nlanes);
        if (nlanes < 1) return fail(ctx, DEFTRI_E_HIP, "lane allocation failed: " + ctx->err);
    }
    R.lanes = nlanes;
    // PCG steps; after kPcgGiveUp consecutive fallbacks in one call the remaining trials go straight
    // to the LDL^T (small, weakly damped problems where CG cannot win: their steps take thousands of
    // iterations); deterministic, the same problem always takes the same path
    bool pcg = nlanes == 1 && use_pcg(ctx);
    int consec_fallbacks = 0;
    constexpr int kPcgGiveUp = 2;
    for (it = 0; it < prm->n_iterations; it++) {
        hipEventRecord(ctx->ev[0], ctx->st);
        if ((rc = eval_chi2_dev(ctx, true, analytic, 0))) return rc;   // computeActiveErrors + linearizeOplus
        build_system(ctx, pcg, it == 0);                    // buildSystem
        if (it == 0) {
            if (dist) {                                      // max of the rank-summed diagonal
                launch_diag_entries(L, ctx->d_diagv, ctx->st);
                if ((rc = dist_allreduce(ctx, ctx->d_diagv, L.ndof, 0))) return rc;
                launch_absmax(L.ndof, ctx->d_diagv, ctx->d_part, kRedParts, ctx->d_scal + 2, ctx->st);
            } else if (!ctx->assembled) {                    // matrix-free: the diagonal from k_mf_lin
                launch_absmax(L.ndof, ctx->G.mf_dvec, ctx->d_part, kRedParts, ctx->d_scal + 2, ctx->st);
            } else {
                launch_maxdiag(L, ctx->d_part, kRedParts, ctx->d_scal + 2, ctx->st);
            }
        }
        hipEventRecord(ctx->ev[1], ctx->st);
        double *chis = ctx->hpin;           // pinned: a pageable readback costs ~100 us per call
        HIPOK(hipMemcpyAsync(chis, ctx->d_scal, sizeof(double) * 3, hipMemcpyDeviceToHost, ctx->st));
        // only iteration 0 needs a value before its first trial (lambda from max diag); later
        // iterations read this iteration's chi2 with the first trial's (or round's) scalars
        bool chi_pending = true;
        if (it == 0) {
            HIPOK(hipStreamSynchronize(ctx->st));
            t_lin += ev_ms(ctx, 0, 1);
            currentChi = chis[0];
            chi_pending = false;
            lambda = prm->user_lambda > 0 ? prm->user_lambda : tau * chis[2];
            ni = 2;
        }
        double rho = 0;
        int qmax = 0;
        bool restore_pending = false;                        // a rejected fused trial's state not yet restored
        if (nlanes > 1) {
            // speculative rounds: lanes 0..nl-1 run trials qmax..qmax+nl-1 concurrently; the host then
            // replays g2o's accept/reject sequence over their scalars in trial order
            bool done = false;
            while (!done) {
                const int nl = std::min(nlanes, max_trials - qmax);
                double lam[kMaxLanes];
                double lc = lambda, nc = ni;
                for (int t = 0; t < nl; t++) { lam[t] = lc; lc *= nc; nc *= 2; }
                hipEventRecord(ctx->ev[2], ctx->st);
                lanes_round(ctx, nl, lam, analytic);
                hipEventRecord(ctx->ev[5], ctx->st);
                HIPOK(hipStreamSynchronize(ctx->st));       // the one host round trip of a round
                if (chi_pending) { currentChi = chis[0]; chi_pending = false; t_lin += ev_ms(ctx, 0, 1); }
                t_fac += ev_ms(ctx, 2, 5);
                R.trials_executed += nl;
                int acc = -1;
                for (int t = 0; t < nl; t++)
                    if (ctx->lane_ipin[t] & kStatusWaitTimeout)
                        return fail(ctx, DEFTRI_E_HIP, "factorization: a fused TRSM tile timed out waiting for its panel");
                for (int t = 0; t < nl && !done; t++) {
                    const bool ok2 = ctx->lane_ipin[t] == 0;
                    double tempChi = ok2 ? ctx->lane_pin[2 * t] : std::numeric_limits<double>::max();
                    rho = (currentChi - tempChi);
                    double scale = ctx->lane_pin[2 * t + 1] + 1e-3;
                    rho /= scale;
                    R.trials_total++;
                    if (rho > 0 && std::isfinite(tempChi)) {
                        double alpha = 1. - std::pow((2 * rho - 1), 3);
                        alpha = std::min(alpha, 2. / 3.);
                        double scaleFactor = std::max(1. / 3., alpha);
                        lambda *= scaleFactor;
                        ni = 2;
                        currentChi = tempChi;
                        acc = t;
                    } else {
                        lambda *= ni;
                        ni *= 2;
                        R.trials_rejected++;
                    }
                    qmax++;
                    // g2o: `if (!g2o_isfinite(_currentLambda)) break;` after a rejected trial
                    if (!(rho < 0 && qmax < max_trials) || !std::isfinite(lambda)) done = true;
                }
                if (acc >= 0) adopt_lane_state(ctx, acc);
            }
        } else do {
            // PCG trials on one rank: the prologue (state backup, flag and PCG records cleared) and
            // the read-back (scalars, flag, the solve's record) are one launch each
            const bool fused = pcg && !dist;
            if (fused) {
                // after a rejected trial the prologue restores the state from the backup instead
                pcg_limits(ctx);
                launch_trial_begin(P, L.flag, ctx->G.rec, (int64_t)kPcgRec * (ctx->G.max_it + 2), ctx->st,
                                   restore_pending);
                restore_pending = false;
            } else {
                if (restore_pending) { pop_state(ctx); restore_pending = false; }   // PCG just given up
                push_state(ctx);
                HIPOK(hipMemsetAsync(L.flag, 0, sizeof(int), ctx->st));
            }
            double *sc = ctx->hpin + 4;
            // the trial's evaluation: _optimizer->update(x) (skipped on a zero pivot), chi2, rho's
            // denominator, read-backs (one host round trip); rec_j: the PCG record read back with them
            auto evaluate = [&](const double *rec_j) -> int {
                trial_ev(ctx, ctx->ev[4], ctx->st);
                launch_update_state(P, ctx->d_dx, ctx->st, L.flag);
                if (dist) {
                    // chi2 of the rank's edges, dx.(lambda dx + b) with b partial and lambda once per dof,
                    // the zero-pivot flag: one all-reduce of the three (a zero pivot on any rank rejects)
                    int r2 = eval_chi2_dev(ctx, false, analytic, 0, false);
                    if (r2) return r2;
                    launch_sum(ctx->S.ndof, ctx->d_dx, L.b, lambda, 3, ctx->d_part, kRedParts, ctx->d_scal + 1, ctx->st,
                               ctx->d_dofw);
                    launch_int_to_double(1, L.flag, ctx->d_scal + 2, ctx->st);
                    if ((r2 = dist_allreduce(ctx, ctx->d_scal, 3, 0))) return r2;
                    trial_ev(ctx, ctx->ev[5], ctx->st);
                    HIPOK(hipMemcpyAsync(sc, ctx->d_scal, sizeof(double) * 3, hipMemcpyDeviceToHost, ctx->st));
                } else {
                    // computeActiveErrors; activeRobustChi2; rho's denominator dx.(lambda dx + b)
                    SumJob den;
                    den.n = ctx->S.ndof; den.a = ctx->d_dx; den.b = L.b; den.lambda = lambda; den.mode = 1;
                    den.out = ctx->d_scal + 1;
                    eval_chi2_dev(ctx, false, analytic, 0, true, &den);
                    trial_ev(ctx, ctx->ev[5], ctx->st);
                    if (fused) {
                        launch_trial_readback(ctx->d_scal, 2, L.flag, rec_j, kPcgRec, sc, ctx->ipin, ctx->hpin + 16,
                                              ctx->st);
                    } else {
                        HIPOK(hipMemcpyAsync(sc, ctx->d_scal, sizeof(double) * 2, hipMemcpyDeviceToHost, ctx->st));
                        HIPOK(hipMemcpyAsync(ctx->ipin, L.flag, sizeof(int), hipMemcpyDeviceToHost, ctx->st));
                    }
                }
                return 0;
            };
            bool solved = false, evaluated = false;
            trial_ev(ctx, ctx->ev[2], ctx->st);
            if (pcg) {
                // PCG step with the evaluation queued behind the predicted iteration count: when the
                // solve has converged by then, the trial costs one round trip; otherwise the state
                // is restored, the solve continues (or falls back) and the evaluation is redone
                auto t0 = std::chrono::steady_clock::now();
                int j = 0, its = 0;
                pcg_start(ctx, lambda, L.b, j, fused);
                trial_ev(ctx, ctx->ev[3], ctx->st);
                if ((rc = evaluate(fused ? ctx->G.rec + (size_t)kPcgRec * (j + 1) : nullptr))) return rc;
                if (!fused && (rc = pcg_fetch(ctx, j))) return rc;
                HIPOK(hipStreamSynchronize(ctx->st));
                const int v = pcg_verdict(ctx, j, its);
                if (v > 0) {
                    solved = evaluated = true;
                } else {
                    pop_state(ctx);
                    if (v == 0 && (rc = pcg_poll(ctx, lambda, j, solved, its))) return rc;
                }
                R.ms_pcg += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                R.pcg_iterations += its;
                if (solved) { R.pcg_trials++; consec_fallbacks = 0; }
                else R.pcg_fallbacks++;
                if (!solved && ++consec_fallbacks >= kPcgGiveUp) { pcg = false; R.pcg_given_up = 1; }
                if (prm->verbose)
                    std::fprintf(stderr, "[deftri] pcg lambda %.6e iterations %d %s\n", lambda, its, solved ? "converged" : "-> LDL^T");
                if (!solved) trial_ev(ctx, ctx->ev[2], ctx->st);
            }
            if (!solved) {
                ensure_assembled(ctx);                       // a matrix-free PCG step left H unassembled
                ctx->hpin[12] = lambda;                      // pinned: read by the copy at its turn in the stream
                HIPOK(hipMemcpyAsync(ctx->d_lam, ctx->hpin + 12, sizeof(double), hipMemcpyHostToDevice, ctx->st));
                if (launch_trial_graph(ctx)) {
                    trial_ev(ctx, ctx->ev[3], ctx->st);     // factor + solve in one graph: timed as factor
                } else {
                    launch_scatter(L, lambda, ctx->st);      // setLambda
                    launch_factor(L, ctx->st, ctx->side, ctx->sync_ev, 64, hook, ctx);
                    trial_ev(ctx, ctx->ev[3], ctx->st);
                    ctx->hook_x = ctx->d_dx;
                    launch_solve(L, L.b, ctx->d_dx, ctx->st, dist ? L.b : nullptr, hook, ctx);
                    if (ctx->hook_rc) return ctx->hook_rc;
                }
            }
            if (solved && !evaluated) trial_ev(ctx, ctx->ev[3], ctx->st);
            if (!evaluated && (rc = evaluate(nullptr))) return rc;
            HIPOK(hipStreamSynchronize(ctx->st));       // the one host round trip of a trial
            if (chi_pending) { currentChi = chis[0]; chi_pending = false; t_lin += ev_ms(ctx, 0, 1); }
            if (dist ? sc[2] >= kStatusWaitTimeout : (*ctx->ipin & kStatusWaitTimeout) != 0)
                return fail(ctx, DEFTRI_E_HIP, "factorization: a fused TRSM tile timed out waiting for its panel");
            const bool ok2 = dist ? sc[2] == 0.0 : *ctx->ipin == 0;
            if (trial_events_on()) { t_fac += ev_ms(ctx, 2, 3); t_sol += ev_ms(ctx, 3, 4); t_upd += ev_ms(ctx, 4, 5); }
            double tempChi = ok2 ? sc[0] : std::numeric_limits<double>::max();
            rho = (currentChi - tempChi);
            double scale = sc[1] + 1e-3;
            rho /= scale;
            R.trials_total++;
            R.trials_executed++;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                double scaleFactor = std::max(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                if (fused) restore_pending = true;           // the next prologue (or the loop's end) restores
                else pop_state(ctx);
                R.trials_rejected++;
                if (!std::isfinite(lambda)) { qmax++; break; }   // g2o OptimizationAlgorithmLevenberg::solve
            }
            qmax++;
        } while (rho < 0 && qmax < max_trials);
        if (restore_pending) { pop_state(ctx); restore_pending = false; }
        if (it < DEFTRI_MAX_REPORT_ITERS) { R.chi2_iter[it] = currentChi; R.trials_iter[it] = qmax; }
        if (prm->verbose)
            std::fprintf(stderr, "[deftri] it %d chi2 %.9e lambda %.6e trials %d\n", it, currentChi, lambda, qmax);
        if (qmax == max_trials || rho == 0 || !std::isfinite(lambda)) { status = DEFTRI_STATUS_TERMINATE; it++; break; }
    }
    if ((rc = eval_chi2_dev(ctx, false, analytic, 0))) return rc;
    R.chi2_final = read_scal(ctx, 0);
    HIPOK(hipStreamSynchronize(ctx->st));
    R.status = status;
    R.iterations = it;
    R.lambda_final = lambda;
    R.ms_linearize = t_lin; R.ms_factor = t_fac; R.ms_solve = t_sol; R.ms_update = t_upd;
    if (nlanes == 1 && !trial_events_on()) R.ms_factor = R.ms_solve = R.ms_update = -1.0;   // not measured
    R.plan = DEFTRI_PLAN_MULTIFRONTAL;
    R.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    return 0;
}

int deftri_pixels_stand_dev(deftri_ctx *ctx, const deftri_map *map, deftri_pixels_error *out) {
    if (!ctx || !map || !out || map->n_keyframes < 0 || (map->n_keyframes > 0 && !map->keyframes)) return DEFTRI_E_ARG;
    if (ctx->device < 0) return fail(ctx, DEFTRI_E_NODEVICE, "host-only context");
    hipSetDevice(ctx->device);
    const int K = map->n_keyframes;
    // per keyframe: R (fp32, Eigen toRotationMatrix of the fp32 unit quaternion), t, kb8
    std::vector<float> cams(20 * (size_t)std::max(K, 1));
    for (int k = 0; k < K; k++) {
        const deftri_keyframe &kf = map->keyframes[k];
        float x = (float)kf.pose[0], y = (float)kf.pose[1], z = (float)kf.pose[2], w = (float)kf.pose[3];
        float tx = 2 * x, ty = 2 * y, tz = 2 * z, twx = tx * w, twy = ty * w, twz = tz * w;
        float txx = tx * x, txy = ty * x, txz = tz * x, tyy = ty * y, tyz = tz * y, tzz = tz * z;
        float *c = &cams[20 * (size_t)k];
        c[0] = 1 - (tyy + tzz); c[1] = txy - twz;       c[2] = txz + twy;
        c[3] = txy + twz;       c[4] = 1 - (txx + tzz); c[5] = tyz - twx;
        c[6] = txz - twy;       c[7] = tyz + twx;       c[8] = 1 - (txx + tyy);
        for (int q = 0; q < 3; q++) c[9 + q] = (float)kf.pose[4 + q];
        for (int q = 0; q < 8; q++) c[12 + q] = kf.kb8[q];
    }
    // matches of each pair in the reference's loop order (:386-416)
    std::vector<float> pts, obs;
    std::vector<int32_t> pair_cams, pair_first{0};
    for (int a = 0; a < K; a++)
        for (int b = a + 1; b < K; b++) {
            const deftri_keyframe &k1 = map->keyframes[b], &k2 = map->keyframes[a];
            pair_cams.push_back(b); pair_cams.push_back(a);
            const int n = std::min(k1.n_slots, k2.n_slots);
            for (int i = 0; i < n; i++) {
                if (k1.point_id[i] < 0 || k2.point_id[i] < 0) continue;
                const int o1 = k1.obs_index[i], o2 = k2.obs_index[i];
                if (o1 < 0 || o2 < 0) continue;
                if (o1 >= k1.n_obs || o2 >= k2.n_obs) return fail(ctx, DEFTRI_E_ARG, "observation index out of range");
                for (int q = 0; q < 3; q++) pts.push_back(k1.point_pos[3 * (int64_t)i + q]);
                for (int q = 0; q < 3; q++) pts.push_back(k2.point_pos[3 * (int64_t)i + q]);
                obs.push_back(k1.kp_uv[2 * (int64_t)o1]); obs.push_back(k1.kp_uv[2 * (int64_t)o1 + 1]);
                obs.push_back(k2.kp_uv[2 * (int64_t)o2]); obs.push_back(k2.kp_uv[2 * (int64_t)o2 + 1]);
            }
            pair_first.push_back((int32_t)(pts.size() / 6));
        }
    const int npair = (int)pair_cams.size() / 2;
    std::vector<int32_t> bf, bl, bp;
    for (int p = 0; p < npair; p++)
        for (int32_t s = pair_first[p]; s < pair_first[p + 1]; s += 256) {
            bf.push_back(s); bl.push_back(std::min(s + 256, pair_first[p + 1])); bp.push_back(p);
        }
    const int nblk = (int)bf.size();
    std::vector<double> part(8 * (size_t)std::max(nblk, 1), 0.0);
    if (nblk > 0) {
        // scratch buffers of this call (one allocation, freed before returning)
        const size_t nb_i = 3 * (size_t)nblk + 2 * (size_t)npair, nb_f = cams.size() + pts.size() + obs.size();
        const size_t bytes = 8 * part.size() + 4 * nb_f + 4 * nb_i + 64;
        char *dbuf = nullptr;
        HIPOK(hipMalloc(&dbuf, bytes));
        double *d_part = (double *)dbuf;
        float *d_cams = (float *)(d_part + part.size());
        float *d_pts = d_cams + cams.size(), *d_obs = d_pts + pts.size();
        int32_t *d_bf = (int32_t *)(d_obs + obs.size()), *d_bl = d_bf + nblk, *d_bp = d_bl + nblk, *d_pc = d_bp + nblk;
        hipMemcpyAsync(d_cams, cams.data(), 4 * cams.size(), hipMemcpyHostToDevice, ctx->st);
        hipMemcpyAsync(d_pts, pts.data(), 4 * pts.size(), hipMemcpyHostToDevice, ctx->st);
        hipMemcpyAsync(d_obs, obs.data(), 4 * obs.size(), hipMemcpyHostToDevice, ctx->st);
        hipMemcpyAsync(d_bf, bf.data(), 4 * (size_t)nblk, hipMemcpyHostToDevice, ctx->st);
        hipMemcpyAsync(d_bl, bl.data(), 4 * (size_t)nblk, hipMemcpyHostToDevice, ctx->st);
        hipMemcpyAsync(d_bp, bp.data(), 4 * (size_t)nblk, hipMemcpyHostToDevice, ctx->st);
        hipMemcpyAsync(d_pc, pair_cams.data(), 4 * pair_cams.size(), hipMemcpyHostToDevice, ctx->st);
        launch_pixel_partials(nblk, d_bf, d_bl, d_bp, d_pc, d_cams, d_pts, d_obs, d_part, ctx->st);
        hipMemcpyAsync(part.data(), d_part, 8 * part.size(), hipMemcpyDeviceToHost, ctx->st);
        hipError_t e = hipStreamSynchronize(ctx->st);
        hipFree(dbuf);
        if (e != hipSuccess) return fail(ctx, DEFTRI_E_HIP, std::string("pixels_stand_dev: ") + hipGetErrorString(e));
    }
    // the reference's per-pair formulas (:454-485); meanUV and nMatches carry over pairs
    double mUV1[2] = {0, 0}, mUV2[2] = {0, 0};
    double mC1 = 0, mC2 = 0, dC1 = 0, dC2 = 0;
    size_t nMatches = 0;
    for (int p = 0, blk = 0; p < npair; p++) {
        double sum[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (; blk < nblk && bp[blk] == p; blk++)
            for (int q = 0; q < 8; q++) sum[q] += part[8 * (size_t)blk + q];
        nMatches += (size_t)(pair_first[p + 1] - pair_first[p]);
        const double nm = (double)nMatches;
        for (int q = 0; q < 2; q++) { mUV1[q] += sum[q]; mUV2[q] += sum[4 + q]; }
        for (int q = 0; q < 2; q++) { mUV1[q] /= nm; mUV2[q] /= nm; }
        mC1 = (mUV1[0] + mUV1[1]) / 2.0;
        mC2 = (mUV2[0] + mUV2[1]) / 2.0;
        dC1 = (std::sqrt(sum[2] / nm) + std::sqrt(sum[3] / nm)) / 2.0;
        dC2 = (std::sqrt(sum[6] / nm) + std::sqrt(sum[7] / nm)) / 2.0;
    }
    out->avgc1 = mC1; out->avgc2 = mC2; out->avg = (mC1 + mC2) / 2.0;
    out->desvc1 = dC1; out->desvc2 = dC2; out->desv = (dC1 + dC2) / 2.0;
    return 0;
}

int deftri_triangulate_nrslam(deftri_ctx *ctx, int32_t n, const float *uv1, const float *uv2, const float *kb8_1,
                              const float *kb8_2, const float *T1w, const float *T2w, float min_cos, float *x3d_1,
                              float *x3d_2, uint8_t *valid) {
    if (!ctx || n < 0 || (n > 0 && (!uv1 || !uv2 || !x3d_1 || !x3d_2 || !valid)) || !kb8_1 || !kb8_2 || !T1w || !T2w)
        return DEFTRI_E_ARG;
    if (ctx->device < 0) return fail(ctx, DEFTRI_E_NODEVICE, "host-only context");
    if (n == 0) return 0;
    hipSetDevice(ctx->device);
    // Sophus: T1w.inverse() = [R1^T | -(R1^T t1)], T21 = T2w * T1w.inverse(), T2w.inverse()
    auto inverse = [](const float *T, float *Ti) {
        for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) Ti[4 * i + j] = T[4 * j + i];
        for (int i = 0; i < 3; i++) Ti[4 * i + 3] = -(Ti[4 * i] * T[3] + Ti[4 * i + 1] * T[7] + Ti[4 * i + 2] * T[11]);
    };
    float Tp[48], T1i[12];
    std::memcpy(Tp, T1w, 12 * sizeof(float));
    std::memcpy(Tp + 12, T2w, 12 * sizeof(float));
    inverse(T1w, T1i);
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++)
            Tp[24 + 4 * i + j] = T2w[4 * i] * T1i[j] + T2w[4 * i + 1] * T1i[4 + j] + T2w[4 * i + 2] * T1i[8 + j];
        Tp[24 + 4 * i + 3] = (T2w[4 * i] * T1i[3] + T2w[4 * i + 1] * T1i[7] + T2w[4 * i + 2] * T1i[11]) + T2w[4 * i + 3];
    }
    inverse(T2w, Tp + 36);
    const size_t N = (size_t)n;
    const size_t bytes = 4 * (2 * N + 2 * N + 8 + 8 + 48 + 3 * N + 3 * N) + N + 64;
    char *dbuf = nullptr;
    HIPOK(hipMalloc(&dbuf, bytes));
    float *d_uv1 = (float *)dbuf, *d_uv2 = d_uv1 + 2 * N, *d_k1 = d_uv2 + 2 * N, *d_k2 = d_k1 + 8, *d_T = d_k2 + 8;
    float *d_x1 = d_T + 48, *d_x2 = d_x1 + 3 * N;
    uint8_t *d_v = (uint8_t *)(d_x2 + 3 * N);
    hipMemcpyAsync(d_uv1, uv1, 8 * N, hipMemcpyHostToDevice, ctx->st);
    hipMemcpyAsync(d_uv2, uv2, 8 * N, hipMemcpyHostToDevice, ctx->st);
    hipMemcpyAsync(d_k1, kb8_1, 32, hipMemcpyHostToDevice, ctx->st);
    hipMemcpyAsync(d_k2, kb8_2, 32, hipMemcpyHostToDevice, ctx->st);
    hipMemcpyAsync(d_T, Tp, sizeof(Tp), hipMemcpyHostToDevice, ctx->st);
    launch_triangulate_nrslam(n, d_uv1, d_uv2, d_k1, d_k2, d_T, min_cos, d_x1, d_x2, d_v, ctx->st);
    hipMemcpyAsync(x3d_1, d_x1, 12 * N, hipMemcpyDeviceToHost, ctx->st);
    hipMemcpyAsync(x3d_2, d_x2, 12 * N, hipMemcpyDeviceToHost, ctx->st);
    hipMemcpyAsync(valid, d_v, N, hipMemcpyDeviceToHost, ctx->st);
    hipError_t e = hipStreamSynchronize(ctx->st);
    hipFree(dbuf);
    if (e != hipSuccess) return fail(ctx, DEFTRI_E_HIP, std::string("triangulate: ") + hipGetErrorString(e));
    return 0;
}

int deftri_download(deftri_ctx *ctx, double *points, double *scales, double *tg) {
    if (!ctx || !ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(ctx->device);
    if (ctx->sp_on) { int rc = ctx->sp->download(points, scales, tg); return rc ? fail(ctx, rc, ctx->sp->err) : 0; }
    DevProblem &P = ctx->P;
    if (points) HIPOK(hipMemcpy(points, P.points, sizeof(double) * 3 * (size_t)P.P, hipMemcpyDeviceToHost));
    if (scales) HIPOK(hipMemcpy(scales, P.scales, sizeof(double) * (size_t)P.S, hipMemcpyDeviceToHost));
    if (tg) HIPOK(hipMemcpy(tg, P.tg, sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToHost));
    return 0;
}

int deftri_eval_chi2(deftri_ctx *ctx, double *chi2) {
    if (!ctx || !ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(ctx->device);
    if (ctx->sp_on) { int rc = ctx->sp->chi2(chi2); return rc ? fail(ctx, rc, ctx->sp->err) : 0; }
    eval_chi2_dev(ctx, false, true, 0);
    *chi2 = read_scal(ctx, 0);
    return 0;
}

int deftri_eval_gradient(deftri_ctx *ctx, double *b, double *hdiag, int64_t n) {
    if (ctx && ctx->dist()) return fail(ctx, DEFTRI_E_ARG, "not available on a point-sharded context");
    if (!ctx || !ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    if (ctx->sp_on) {
        hipSetDevice(ctx->device);
        int rc = ctx->sp->gradient(b, hdiag, n, true);   // analytic J, as the multifrontal plan
        return rc ? fail(ctx, rc, ctx->sp->err) : 0;
    }
    if (n != ctx->S.ndof) return fail(ctx, DEFTRI_E_ARG, "size mismatch");
    hipSetDevice(ctx->device);
    eval_chi2_dev(ctx, true, true, 0);
    build_system(ctx, false);
    HIPOK(hipStreamSynchronize(ctx->st));
    if (b) HIPOK(hipMemcpy(b, ctx->L.b, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost));
    if (hdiag) {
        std::vector<double> hv(ctx->S.hval_size);
        HIPOK(hipMemcpy(hv.data(), ctx->L.hval, sizeof(double) * hv.size(), hipMemcpyDeviceToHost));
        // diagonal blocks: column vertex == row vertex
        const Symbolic &S = ctx->S;
        for (int64_t blk = 0; blk < S.nblocks; blk++) {
            if (!S.blk_diag[blk]) continue;
            const int c = S.blk_cols[blk];
            for (int k = 0; k < c; k++) hdiag[S.blk_col_dof[blk] + k] = hv[S.blk_val_off[blk] + k * c + k];
        }
    }
    return 0;
}

int deftri_eval_hessian_product(deftri_ctx *ctx, const double *x, double *y, int64_t n) {
    if (ctx && ctx->dist()) return fail(ctx, DEFTRI_E_ARG, "not available on a point-sharded context");
    if (!ctx || !ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    if (ctx->sp_on) {                        // the iterative plan's own matrix-free product (H never assembled)
        if (!x || !y) return fail(ctx, DEFTRI_E_ARG, "null array");
        hipSetDevice(ctx->device);
        int rc = ctx->sp->hessian_product(0.0, x, y, n);
        return rc ? fail(ctx, rc, ctx->sp->err) : 0;
    }
    if (n != ctx->S.ndof || !x || !y) return fail(ctx, DEFTRI_E_ARG, "size mismatch");
    hipSetDevice(ctx->device);
    double *dx = nullptr, *dy = nullptr;
    HIPOK(hipMalloc(&dx, sizeof(double) * (size_t)n));
    HIPOK(hipMalloc(&dy, sizeof(double) * (size_t)n));
    hipMemcpy(dx, x, sizeof(double) * (size_t)n, hipMemcpyHostToDevice);
    eval_chi2_dev(ctx, true, true, 0);
    build_system(ctx, false);
    launch_hmul(ctx->L, ctx->L.blk_row_dof, ctx->L.blk_col_dof, dx, dy, n, ctx->st);
    hipStreamSynchronize(ctx->st);
    hipMemcpy(y, dy, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost);
    hipFree(dx); hipFree(dy);
    return 0;
}

int deftri_eval_damped_solve(deftri_ctx *ctx, double lambda, const double *rhs, double *x, int64_t n) {
    if (ctx && ctx->dist()) return fail(ctx, DEFTRI_E_ARG, "not available on a point-sharded context");
    if (!ctx || !ctx->have) return fail(ctx, DEFTRI_E_NOPROBLEM, "no problem uploaded");
    if (ctx->sp_on && ctx->lin_solver != DEFTRI_SOLVER_PCG) {
        const int rc0 = ensure_multifrontal(ctx);     // an LDL^T solve asked for
        if (rc0) return rc0;
    }
    if (ctx->sp_on) {
        if (!rhs || !x) return fail(ctx, DEFTRI_E_ARG, "null array");
        hipSetDevice(ctx->device);
        int rc = ctx->sp->damped_solve(lambda, rhs, x, n);
        return rc ? fail(ctx, rc, ctx->sp->err) : 0;
    }
    if (n != ctx->S.ndof || !rhs || !x) return fail(ctx, DEFTRI_E_ARG, "size mismatch");
    hipSetDevice(ctx->device);
    (void)hipGetLastError();                    // the status check below reads this call's errors only
    double *dr = nullptr;
    HIPOK(hipMalloc(&dr, sizeof(double) * (size_t)n));
    hipMemcpy(dr, rhs, sizeof(double) * (size_t)n, hipMemcpyHostToDevice);
    eval_chi2_dev(ctx, true, true, 0);
    build_system(ctx, false);                   // H for the LDL^T; a matrix-free PCG step reads k_mf_lin's
    if (use_pcg(ctx) && ctx->G.mf) launch_mf_lin(ctx->G, false, ctx->st);
    hipMemsetAsync(ctx->L.flag, 0, sizeof(int), ctx->st);
    bool solved = false;
    if (use_pcg(ctx)) {                         // the configured step solver, as deftri_solve_lm uses it
        int its = 0;
        const int rc = pcg_step(ctx, lambda, dr, solved, its);
        if (rc) { hipFree(dr); return rc; }
    }
    if (!solved) {
        launch_scatter(ctx->L, lambda, ctx->st);
        launch_factor(ctx->L, ctx->st, ctx->side, ctx->sync_ev, 64);
        launch_solve(ctx->L, dr, ctx->d_dx, ctx->st);
    }
    int flag = 0;
    hipMemcpyAsync(&flag, ctx->L.flag, sizeof(int), hipMemcpyDeviceToHost, ctx->st);
    hipStreamSynchronize(ctx->st);
    hipMemcpy(x, ctx->d_dx, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost);
    hipFree(dr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(ctx, DEFTRI_E_HIP, hipGetErrorString(e));
    if (flag & kStatusWaitTimeout) return fail(ctx, DEFTRI_E_HIP, "factorization: a fused TRSM tile timed out waiting for its panel");
    return flag ? fail(ctx, DEFTRI_E_NUMERIC, "zero pivot") : 0;
}

// ---------------------------------------------------------------------------------------------
// map level
// ---------------------------------------------------------------------------------------------
}  // extern "C"
namespace {
// a context with a device runs computeR there
GraphDevice *graph_device(deftri_ctx *ctx) {
    if (ctx->device < 0) return nullptr;
    hipSetDevice(ctx->device);
    if (!ctx->gdev) ctx->gdev.reset(new GraphDevice(ctx->device, ctx->st));
    return ctx->gdev.get();
}
}  // namespace
extern "C" {

int deftri_arap_build_graph(deftri_ctx *ctx, const deftri_map *map, double rep_weight, double arap_weight,
                            float depth_error, const deftri_problem_desc **desc_out) {
    if (!ctx || !map || !desc_out) return DEFTRI_E_ARG;
    std::string err;
    if (!build_arap_graph(*map, rep_weight, arap_weight, depth_error, ctx->graph, err, ctx->pair_window, graph_device(ctx)))
        return fail(ctx, DEFTRI_E_GRAPH, err);
    *desc_out = &ctx->graph.desc;
    return 0;
}

int deftri_graph_stats(const deftri_ctx *ctx, int64_t *memo_hits, int64_t *struct_hits, double *ms_last) {
    if (!ctx) return DEFTRI_E_ARG;
    if (memo_hits) *memo_hits = ctx->graph.memo_hits;
    if (struct_hits) *struct_hits = ctx->graph.struct_hits;
    if (ms_last) *ms_last = ctx->graph.ms_last;
    return 0;
}

int deftri_graph_repairs(const deftri_ctx *ctx, int64_t *meshes, int64_t *flips) {
    if (!ctx) return DEFTRI_E_ARG;
    if (meshes) *meshes = ctx->graph.mesh_repairs;
    if (flips) *flips = ctx->graph.mesh_flips;
    return 0;
}

int deftri_arap_graph_point_ids(const deftri_ctx *ctx, int64_t *ids, int64_t n) {
    if (!ctx || !ids) return DEFTRI_E_ARG;
    if (n != (int64_t)ctx->graph.point_mpid.size()) return DEFTRI_E_ARG;
    std::memcpy(ids, ctx->graph.point_mpid.data(), sizeof(int64_t) * (size_t)n);
    return 0;
}

int deftri_arap_optimization(deftri_ctx *ctx, deftri_map *map, double rep_weight, double global_weight,
                             double arap_weight, double alpha, double beta, float depth_error,
                             int32_t n_iterations, double *optimization_update, deftri_report *report) {
    (void)global_weight; (void)alpha; (void)beta;   // stored but unused by the reference edges
    if (!ctx || !map) return DEFTRI_E_ARG;
    static const bool timing = std::getenv("DEFTRI_CALL_TIMING") != nullptr;   // stage times of the call
    const auto t0 = std::chrono::steady_clock::now();
    auto ms_since = [](std::chrono::steady_clock::time_point a) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
    };
    std::string err;
    if (!build_arap_graph(*map, rep_weight, arap_weight, depth_error, ctx->graph, err, ctx->pair_window, graph_device(ctx)))
        return fail(ctx, DEFTRI_E_GRAPH, err);
    const double ms_graph = ms_since(t0);
    const auto t1 = std::chrono::steady_clock::now();
    int rc = deftri_problem_upload(ctx, &ctx->graph.desc);
    if (rc) return rc;
    const double ms_upload = ms_since(t1);
    const auto t2 = std::chrono::steady_clock::now();
    deftri_lm_params prm{};
    prm.n_iterations = n_iterations;
    prm.max_trials = 10;
    prm.tau = 1e-5;
    prm.analytic_jacobians = ctx->analytic_jac;   // 0 (default): g2o numeric ARAP/depth Jacobians, as the reference
    rc = deftri_solve_lm(ctx, &prm, report);
    if (rc) return rc;
    const double ms_lm = ms_since(t2);
    const auto t3 = std::chrono::steady_clock::now();
    const GraphResult &g = ctx->graph;
    std::vector<double> pts(3 * (size_t)g.desc.n_points), sc(g.desc.n_scales), tg(7 * (size_t)g.desc.n_pairs);
    rc = deftri_download(ctx, pts.data(), sc.data(), tg.data());
    if (rc) return rc;
    writeback_arap(*map, g, pts, sc, tg, optimization_update);
    if (timing)
        std::fprintf(stderr, "[deftri call] graph %.1f ms, upload %.1f, LM %.1f, download + write-back %.1f, total %.1f\n", ms_graph,
                     ms_upload, ms_lm, ms_since(t3), ms_since(t0));
    return 0;
}

}  // extern "C"
