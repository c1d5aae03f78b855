// spcg_solver.cpp — g2o-semantics Levenberg–Marquardt on the point-sharded matrix-free PCG plan
// (spcg.h).  The control flow restates OptimizationAlgorithmLevenberg::solve as driven by
// `optimizer.optimize(nOptIterations)` (reference g2oBundleAdjustment.cc:959-962),
// exactly as solver.cpp's deftri_solve_lm does for the multifrontal plan:
//   per iteration: computeActiveErrors + linearizeOplus, buildSystem (here: the rows' diagonal
//   blocks, b and the heavy blocks only), lambda init at iteration 0 (tau * max diag H), then trials
//   { setLambda; solve; update; computeActiveErrors; rho = (chi_cur - chi_new) /
//   (dx.(lambda dx + b) + 1e-3); accept (lambda *= max(1/3, min(2/3, 1-(2rho-1)^3)), ni = 2) or
//   reject (lambda *= ni, ni *= 2, pop) } while rho < 0 && trials < maxTrials.
// A step whose PCG does not converge within the budget (or breaks down) counts as a failed solve,
// as g2o treats a failed linear solve: chi_new = max, the trial is rejected.  There is no
// factorization behind this plan (a 500k x 8-keyframe factor does not fit one GPU).
//
// Sharded (nranks > 1): every rank runs the same control flow on all-reduced scalars: chi2 of its
// owned edges, the heavy H / b, (r.z, r.r) and (p.q + heavy sums) per CG iteration, the trial's
// chi2 and rho denominator; the boundary rows' (z, p) are exchanged after every CG update and x
// after the solve (SpTransport: RCCL on the solver stream or the caller's host callback).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>

#include "host_threads.h"
#include "spcg.h"
#include "ticket.h"

namespace deftri {

void sp_launch_maxdiag_heavy(const SpDev &G, double *out, hipStream_t st);

namespace {
constexpr int kSpMaxIt = 4096;
constexpr int kSpDefaultIt = 1000;
constexpr int kSpRedParts = 512;
constexpr int kSpRecDoubles = 8;
// the host loop's per-trial wait: poll the stream (no interrupt wake-up; the thread waits anyway) —
// DEFTRI_SYNC_BLOCK=1: hipStreamSynchronize
hipError_t stream_wait(hipStream_t st) {
    static const bool block = std::getenv("DEFTRI_SYNC_BLOCK") != nullptr;
    if (block) return hipStreamSynchronize(st);
    // spin for the first ~100 us (a C2 trial is ~0.4 ms, so the wake-up stays immediate), then yield
    // the core between queries, so a rank sharing a node with its transport's threads (gloo, RCCL's
    // proxy) does not hold a core for the whole CG chain
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e;
    int n = 0;
    while ((e = hipStreamQuery(st)) == hipErrorNotReady) {
        if ((++n & 63) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(100))
            std::this_thread::yield();
    }
    return e;
}

// workgroups per job of the fused chi2 sums: every one takes a ticket on one counter, so fewer, larger
// chunks.  C2 under rocprofv3 (profiles/r03sp_sum_parts.json): 64 parts 11.1 us, 128 12.9, 256 18.5,
// 512 27.9 — every workgroup's ticket costs more than its share of the sum saves
constexpr int kSumParts = 64;
static_assert(kSumParts <= kSpRedParts, "sum parts");

void quat_norm(double *q) {      // SE3Quat::normalizeRotation
    if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
    const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int k = 0; k < 4; k++) q[k] /= n;
}

void quat_mat(const double *q, double *R) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
}  // namespace

#define SPOK(expr)                                                                                  \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess) return fail(DEFTRI_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

SpSolver::SpSolver(int device, hipStream_t st, int rank, int nranks, SpTransport *tr, bool force_sharded)
    : dev_(device), st_(st), rank_(rank), nranks_(nranks), tr_(tr), shard_(nranks > 1 || (force_sharded && tr)) {
    hipHostMalloc((void **)&hpin, 32 * sizeof(double), hipHostMallocDefault);
    hipHostMalloc((void **)&ipin, 16 * sizeof(int), hipHostMallocDefault);
    for (int i = 0; i < 32; i++) hpin[i] = 0.0;
}

SpSolver::~SpSolver() {
    hipSetDevice(dev_);
    hipStreamSynchronize(st_);
    if (cs_) {
        hipStreamSynchronize(cs_);
        hipStreamDestroy(cs_);
    }
    if (ev_upd_) hipEventDestroy(ev_upd_);
    if (ev_halo_) hipEventDestroy(ev_halo_);
    for (void *p : allocs_) hipFree(p);
    if (hpin) hipHostFree(hpin);
    if (h_epart_) hipHostFree(h_epart_);
    if (h_lpart_) hipHostFree(h_lpart_);
    if (ipin) hipHostFree(ipin);
    if (h_snap) hipHostFree(h_snap);
}

template <class T>
int SpSolver::alloc(T **p, int64_t n) {
    *p = nullptr;
    if (n <= 0) n = 1;
    void *v = nullptr;
    hipError_t e = hipMalloc(&v, sizeof(T) * (size_t)n);
    if (e != hipSuccess) return fail(DEFTRI_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    allocs_.push_back(v);
    *p = (T *)v;
    return 0;
}

template <class T>
int SpSolver::put(T **p, const std::vector<T> &v) {
    int rc = alloc(p, (int64_t)v.size());
    if (rc) return rc;
    if (!v.empty()) SPOK(hipMemcpy(*p, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
    return 0;
}

int SpSolver::budget() const { return std::min(kSpMaxIt, max_it > 0 ? max_it : kSpDefaultIt); }

// the state at solve_lm's entry, which an error restores (hand_off_timeout)
int SpSolver::save_entry() {
    SPOK(hipMemcpyAsync(d_entry[0], P.points, sizeof(double) * 3 * (size_t)P.P, hipMemcpyDeviceToDevice, st_));
    SPOK(hipMemcpyAsync(d_entry[1], P.scales, sizeof(double) * (size_t)P.S, hipMemcpyDeviceToDevice, st_));
    SPOK(hipMemcpyAsync(d_entry[2], P.tg, sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToDevice, st_));
    return 0;
}

// a merged-chain alpha hand-off that timed out (spcg.hip m2_alpha_wait): the state the call started
// from is restored (iterations it accepted before the fault are undone, so a retry is a clean run),
// the context switches to the separate alpha launch and the call fails — a device scheduling fault,
// not a numeric verdict, so it never becomes a rejected trial
int SpSolver::hand_off_timeout() {
    G.alpha_kernel = 1;
    hipStreamSynchronize(st_);
    if (in_lm_) {                  // (a bare damped solve does not move the state)
        hipMemcpyAsync(P.points, d_entry[0], sizeof(double) * 3 * (size_t)P.P, hipMemcpyDeviceToDevice, st_);
        hipMemcpyAsync(P.scales, d_entry[1], sizeof(double) * (size_t)P.S, hipMemcpyDeviceToDevice, st_);
        hipMemcpyAsync(P.tg, d_entry[2], sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToDevice, st_);
        hipStreamSynchronize(st_);
    }
    return fail(DEFTRI_E_HIP, "merged CG chain: the alpha hand-off timed out (phase 2's workgroup 0 not resident); "
                              "the state is restored to the call's start and the context now launches alpha "
                              "separately — retry the call");
}

// the values of a problem in the plan's layout (points in row order, the rank's edges): everything
// a structurally identical problem can change
void SpSolver::gather_values(const deftri_problem_desc &d, SpValues &v) const {
    const int32_t NP = d.n_points, Q = d.n_pairs, S = d.n_scales, C = d.n_cams;
    // (the long gathers on host threads: disjoint output ranges)
    v.pts.resize(3 * (size_t)NP);
    chunked(NP, 1 << 16, [&](int, int64_t lo, int64_t hi) {
        for (int64_t r = lo; r < hi; r++)
            for (int c = 0; c < 3; c++) v.pts[3 * (size_t)r + c] = d.points[3 * (size_t)H.point_of_row[r] + c];
    });
    v.tg.assign(d.tg, d.tg + 7 * (size_t)Q);
    v.sc.assign(d.scales, d.scales + S);
    for (int32_t q = 0; q < Q; q++) quat_norm(&v.tg[7 * (size_t)q]);
    v.cpose.assign(d.cam_pose, d.cam_pose + 7 * (size_t)C);
    v.camR.assign(9 * (size_t)std::max(C, 1), 0.0);
    for (int32_t c = 0; c < C; c++) { quat_norm(&v.cpose[7 * (size_t)c]); quat_mat(&v.cpose[7 * (size_t)c], &v.camR[9 * (size_t)c]); }
    v.kb8.assign(d.cam_kb8, d.cam_kb8 + 8 * (size_t)C);
    const size_t nr = H.rep_ids.size(), nd = H.dep_ids.size(), nloc = H.arap_ids.size();
    v.ro.resize(2 * nr); v.ri.resize(nr); v.dm.resize(nd); v.di.resize(nd); v.aw.resize(nloc);
    chunked((int64_t)nr, 1 << 16, [&](int, int64_t lo, int64_t hi) {
        for (int64_t j = lo; j < hi; j++) {
            const int32_t e = H.rep_ids[j];
            v.ro[2 * j] = d.rep_obs[2 * (size_t)e]; v.ro[2 * j + 1] = d.rep_obs[2 * (size_t)e + 1]; v.ri[j] = d.rep_info[e];
        }
    });
    chunked((int64_t)nd, 1 << 16, [&](int, int64_t lo, int64_t hi) {
        for (int64_t j = lo; j < hi; j++) { const int32_t e = H.dep_ids[j]; v.dm[j] = d.dep_meas[e]; v.di[j] = d.dep_info[e]; }
    });
    chunked((int64_t)nloc, 1 << 16, [&](int, int64_t lo, int64_t hi) {
        for (int64_t le = lo; le < hi; le++) v.aw[le] = d.arap_w[H.arap_ids[le]];
    });
    v.rot.resize(9 * H.rot_ids.size());
    chunked((int64_t)H.rot_ids.size(), 1 << 16, [&](int, int64_t lo, int64_t hi) {
        for (int64_t k = lo; k < hi; k++) std::memcpy(&v.rot[9 * k], d.rot + 9 * (size_t)H.rot_ids[k], 9 * sizeof(double));
    });
    v.parea.assign(d.pair_area, d.pair_area + Q);
    v.pinfo.assign(d.pair_info, d.pair_info + Q);
}

// a problem with the uploaded one's structure (same counts and index arrays): copy its values into
// the existing buffers; the plan, the wave layout and every allocation stay
int SpSolver::refresh(const deftri_problem_desc &d) {
    if (!have_) return fail(DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(dev_);
    SPOK(hipStreamSynchronize(st_));
    SpValues v;
    gather_values(d, v);
    auto cp = [&](auto *dst, const auto &src) -> hipError_t {
        return src.empty() ? hipSuccess : hipMemcpyAsync(dst, src.data(), sizeof(src[0]) * src.size(), hipMemcpyHostToDevice, st_);
    };
    SPOK(cp(P.points, v.pts)); SPOK(cp(P.scales, v.sc)); SPOK(cp(P.tg, v.tg));
    SPOK(cp(init_[0], v.pts)); SPOK(cp(init_[1], v.sc)); SPOK(cp(init_[2], v.tg));
    SPOK(cp(P.cam_kb8, v.kb8)); SPOK(cp(P.cam_pose, v.cpose)); SPOK(cp(P.cam_R, v.camR));
    SPOK(cp(P.rep_obs, v.ro)); SPOK(cp(P.rep_info, v.ri)); SPOK(cp(P.dep_meas, v.dm)); SPOK(cp(P.dep_info, v.di));
    SPOK(cp(P.arap_w, v.aw)); SPOK(cp(P.rot, v.rot)); SPOK(cp(P.pair_area, v.parea)); SPOK(cp(P.pair_info, v.pinfo));
    P.huber_delta = d.huber_delta;
    SPOK(hipStreamSynchronize(st_));
    return 0;
}

int SpSolver::upload(const deftri_problem_desc &d) {
    hipSetDevice(dev_);
    hipStreamSynchronize(st_);
    for (void *p : allocs_) hipFree(p);
    allocs_.clear();
    d_lm = nullptr; d_chi_it = nullptr; d_trials_it = nullptr;
    have_ = false;
    P = DevProblem();
    G = SpDev();
    static const bool timing = std::getenv("DEFTRI_UPLOAD_TIMING") != nullptr;
    const auto tu0 = std::chrono::steady_clock::now();
    // tile mode (spcg_tile.cpp: the fused product, every ARAP edge read once per CG iteration), one
    // keyframe pair: one rank on the merged chain from kSpMergeMinDof unknowns, and every sharded
    // context on the single-reduction chain (the product on z there); DEFTRI_SP_NO_TILE=1 keeps the
    // two-phase product everywhere, DEFTRI_SP_SD_NO_TILE=1 on sharded contexts
    static const bool no_tile = std::getenv("DEFTRI_SP_NO_TILE") != nullptr;
    static const bool sd_no_tile = std::getenv("DEFTRI_SP_SD_NO_TILE") != nullptr;
    const int64_t ndof_ = 6 * (int64_t)d.n_pairs + d.n_scales + 3 * (int64_t)d.n_points;
    const bool want_tile = !no_tile && (d.n_pairs == 1 || !shard_) &&
                           (shard_ ? !sd_no_tile
                                   : !std::getenv("DEFTRI_SP_NO_FUSE") && !std::getenv("DEFTRI_SP_NO_MERGE") &&
                                         (ndof_ >= kSpMergeMinDof || std::getenv("DEFTRI_SP_MERGE")));
    const bool planned = build_sp_plan(d, rank_, nranks_, fp32_jac != 0, H, err, want_tile);
    if (before_alloc) {
        before_alloc();
        before_alloc = nullptr;
    }
    if (!planned) return DEFTRI_E_ARG;
    const auto tu1 = std::chrono::steady_clock::now();
    struct Report {                 // DEFTRI_UPLOAD_TIMING=1: plan build vs the rest of the upload
        bool on; std::chrono::steady_clock::time_point a, b;
        ~Report() {
            if (on)
                std::fprintf(stderr, "[deftri upload] plan %.1f ms, values + allocations + copies %.1f ms\n",
                             std::chrono::duration<double, std::milli>(b - a).count(),
                             std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - b).count());
        }
    } rep_{timing, tu0, tu1};
    const int32_t NP = d.n_points, Q = d.n_pairs, S = d.n_scales, C = d.n_cams;
    const int64_t nloc = (int64_t)H.arap_ids.size();
    const int32_t nown = H.hi - H.lo;
    SpValues v;
    gather_values(d, v);
    std::vector<double> &pts = v.pts, &tg = v.tg, &sc = v.sc, &cpose = v.cpose, &camR = v.camR;
    std::vector<float> &kb8 = v.kb8;
    // the rank's edges: structure (rows, cameras, scales, pairs) in the plan's numbering
    const size_t nr = H.rep_ids.size(), nd = H.dep_ids.size();
    std::vector<int32_t> rp(nr), rc(nr), dp(nd), ds(nd), dc(nd);
    chunked((int64_t)nr, 1 << 16, [&](int, int64_t lo, int64_t hi) {
        for (int64_t j = lo; j < hi; j++) { const int32_t e = H.rep_ids[j]; rp[j] = H.row_of_point[d.rep_point[e]]; rc[j] = d.rep_cam[e]; }
    });
    chunked((int64_t)nd, 1 << 16, [&](int, int64_t lo, int64_t hi) {
        for (int64_t j = lo; j < hi; j++) {
            const int32_t e = H.dep_ids[j];
            dp[j] = H.row_of_point[d.dep_point[e]]; ds[j] = d.dep_scale[e]; dc[j] = d.dep_cam[e];
        }
    });
    std::vector<int32_t> apts(4 * (size_t)nloc), apair(nloc);
    chunked(nloc, 1 << 16, [&](int, int64_t lo, int64_t hi) {
        for (int64_t le = lo; le < hi; le++) {
            const int64_t e = H.arap_ids[le];
            for (int k = 0; k < 4; k++) apts[4 * le + k] = H.row_of_point[d.arap_pts[4 * e + k]];
            apair[le] = d.arap_pair[e];
        }
    });
    std::vector<double> &ro = v.ro, &ri = v.ri, &dm = v.dm, &di = v.di, &aw = v.aw, &rot = v.rot, &parea = v.parea,
                        &pinfo = v.pinfo;
    int rc_;
#define PUT(dst, v) if ((rc_ = put(&(dst), v))) return rc_
#define ALLOC(dst, n) if ((rc_ = alloc(&(dst), n))) return rc_
    P.P = NP; P.Q = Q; P.S = S; P.C = C;
    P.R = (int32_t)nr; P.D = (int32_t)nd; P.E = (int32_t)nloc; P.NR = (int32_t)H.rot_ids.size();
    P.huber_delta = d.huber_delta;
    P.jarap_ld = std::max<int64_t>(nloc, 1);        // column-major J: each of the 18 columns coalesced
    PUT(P.points, pts); PUT(P.scales, sc); PUT(P.tg, tg);
    ALLOC(P.points_bak, 3 * (int64_t)NP); ALLOC(P.scales_bak, S); ALLOC(P.tg_bak, 7 * (int64_t)Q);
    ALLOC(d_entry[0], 3 * (int64_t)NP); ALLOC(d_entry[1], S); ALLOC(d_entry[2], 7 * (int64_t)Q);
    PUT(P.cam_kb8, kb8); PUT(P.cam_pose, cpose); PUT(P.cam_R, camR);
    PUT(P.rep_point, rp); PUT(P.rep_cam, rc); PUT(P.rep_obs, ro); PUT(P.rep_info, ri);
    PUT(P.dep_point, dp); PUT(P.dep_scale, ds); PUT(P.dep_cam, dc); PUT(P.dep_meas, dm); PUT(P.dep_info, di);
    PUT(P.arap_pts, apts); PUT(P.arap_pair, apair); PUT(P.arap_rot, H.arap_rot_local); PUT(P.arap_w, aw);
    PUT(P.rot, rot); PUT(P.pair_area, parea); PUT(P.pair_info, pinfo);
    ALLOC(P.Jrep, 6 * (int64_t)nr); ALLOC(P.Wrep, nr); ALLOC(P.Erep, 2 * (int64_t)nr); ALLOC(P.chi_rep, nr);
    ALLOC(P.Jdep, 4 * (int64_t)nd); ALLOC(P.Wdep, nd); ALLOC(P.Edep, nd); ALLOC(P.chi_dep, nd);
    ALLOC(P.Jarap, 18 * std::max<int64_t>(nloc, 1)); ALLOC(P.Warap, nloc); ALLOC(P.Earap, nloc); ALLOC(P.chi_arap, nloc);
    ALLOC(P.tg_pre, 12 * 13 * (int64_t)std::max(Q, 1));
    init_.assign(3, nullptr);
    PUT(init_[0], pts); PUT(init_[1], sc); PUT(init_[2], tg);
    pts.clear(); pts.shrink_to_fit();
    apts.clear(); apts.shrink_to_fit();

    // plan
    G.P = NP; G.Q = Q; G.S = S;
    G.hd = H.hd;
    G.ndof = H.hd + 3 * (int64_t)NP;
    G.row0 = H.lo; G.nown = nown;
    G.nblk = (int32_t)(H.blk.size() / 4);
    G.nrb = (nown + kSpBlock - 1) / kSpBlock;
    G.include_heavy = rank_ == 0 ? 1 : 0;
    int32_t *blk, *hvb, *dperm, *inc, *roff, *doff;
    int64_t *hvbo, *inco;
    PUT(blk, H.blk); PUT(hvb, H.hv_blk); PUT(hvbo, H.hv_blk_off); PUT(dperm, H.dperm);
    PUT(inc, H.inc); PUT(inco, H.inc_off); PUT(roff, H.rep_off); PUT(doff, H.dep_off);
    G.blk = reinterpret_cast<const int4 *>(blk);
    {
        // k_sp_glin_blocks' groups: up to kSpGlinGroup consecutive owned ARAP blocks of one pair with
        // contiguous edges per workgroup (its 27 sums reduced once per group, not per 256 edges); any
        // other block alone
        const int gmax = kSpGlinGroup;
        std::vector<int32_t> gl;
        const int32_t nb = (int32_t)(H.blk.size() / 4);
        for (int32_t b = 0; b < nb;) {
            const int32_t *d0 = &H.blk[4 * (size_t)b];
            const bool arap_owned = (d0[0] & 0xff) == SP_ARAP && (d0[0] >> 8) != 0;
            int32_t n = 1;
            while (arap_owned && n < gmax && b + n < nb) {
                const int32_t *dn = &H.blk[4 * (size_t)(b + n)], *dp = dn - 4;
                if (dn[0] != d0[0] || dn[1] != d0[1] || dn[2] != dp[3]) break;
                n++;
            }
            gl.push_back(b);
            gl.push_back(n);
            b += n;
        }
        int32_t *glb;
        PUT(glb, gl);
        G.glb = reinterpret_cast<const int2 *>(glb);
        G.nglb = (int32_t)(gl.size() / 2);
    }
    G.hv_blk = hvb; G.hv_blk_off = hvbo; G.dperm = dperm;
    G.inc = inc; G.inc_off = inco; G.rep_off = roff; G.dep_off = doff;
    G.apts = P.arap_pts; G.apair = P.arap_pair;
    G.Ja = P.Jarap; G.Wa = P.Warap; G.Ea = P.Earap;
    G.pinfo = P.pair_info;
    G.Jr = P.Jrep; G.Wr = P.Wrep; G.Er = P.Erep;
    G.Jd = P.Jdep; G.Wd = P.Wdep; G.Ed = P.Edep;
    G.dsc = P.dep_scale; G.drow = P.dep_point;
    G.jld = P.jarap_ld;
    if (fp32_jac) { float *j32; ALLOC(j32, 18 * G.jld); G.Ja32 = j32; }
    G.nwaves = (int32_t)(H.woff.size() - 1);
    G.nslots = H.woff.back();
    G.heavy_split = H.max_heavy_blocks > kSpHeavySplit ? 1 : 0;
    {
        // phase-2 row split (DEFTRI_SP_ROW_SPLIT = 1, 2 or 4)
        static const int rs_env = [] {
            const char *e = std::getenv("DEFTRI_SP_ROW_SPLIT");
            const int v = e ? std::atoi(e) : kSpRowSplit;
            return v == 1 || v == 2 || v == 4 ? v : kSpRowSplit;
        }();
        G.rs = rs_env;
        static const int u_env = [] {
            const char *e = std::getenv("DEFTRI_SP_P2_STEP");
            const int v = e ? std::atoi(e) : kSpP2Step;
            return v == 4 || v == 6 || v == 8 ? v : kSpP2Step;
        }();
        G.p2u = u_env;
        static const int g_env = [] {
            const char *e = std::getenv("DEFTRI_SP_GLIN_STEP");
            const int v = e ? std::atoi(e) : kSpGlinStep;
            return v == 4 || v == 6 || v == 8 ? v : kSpGlinStep;
        }();
        G.glu = g_env;
        const int rpw = 4 / G.rs;
        G.nrb2 = (G.nwaves + rpw - 1) / rpw;
    }
    {
        static const bool no_fuse = std::getenv("DEFTRI_SP_NO_FUSE") != nullptr;
        const int64_t heavy_parts = H.hv_blk_off.empty() ? 0 : H.hv_blk_off.back();
        G.fuse = (!shard_ && !no_fuse) ? 1 : 0;
        G.fuse_heavy = (G.fuse && heavy_parts <= kSpFuseHeavyMax && Q + S <= 64) ? 1 : 0;
        // one rank, from kSpMergeMinDof unknowns: two launches per CG iteration (merged chain; alpha
        // from p.Ap).  Smaller problems keep the three-launch chain (alpha from p.q): they are the
        // badly conditioned ones here (thousands of CG iterations per step), where the two alpha
        // formulas' rounding differences can move a solve past its budget, and a CG iteration costs
        // microseconds either way.  DEFTRI_SP_NO_MERGE=1 / DEFTRI_SP_MERGE=1 force either chain.
        static const bool no_merge = std::getenv("DEFTRI_SP_NO_MERGE") != nullptr;
        static const bool force_merge = std::getenv("DEFTRI_SP_MERGE") != nullptr;
        G.merged = (G.fuse && !no_merge && Q + S <= 4096 && (force_merge || G.ndof >= kSpMergeMinDof)) ? 1 : 0;
        G.m_nx = 8 * ((G.nrb + 1 + 7) / 8);
        G.m_nh = 8 * ((Q + S + 7) / 8);
        G.alpha_kernel = 0;                        // (1 after a hand-off timeout: hand_off_timeout)
        // tests: every waiter of this CG iteration's alpha hand-off times out (the error path)
        static const int inj = std::getenv("DEFTRI_SP_INJECT_TIMEOUT_IT") ? std::atoi(std::getenv("DEFTRI_SP_INJECT_TIMEOUT_IT")) : -1;
        G.inj_timeout_it = inj;
        // sharded: the single-reduction chain (3 launches + one all-reduce per CG iteration)
        G.sd = shard_ ? 1 : 0;
        if (G.sd) G.m_nh = 8 * ((Q + S + 2 + 7) / 8);   // + the z.Az and (r.z, r.r) workgroups
    }
    {
        int32_t *rm, *pm, *pi;
        int64_t *wo;
        uint8_t *ws;
        PUT(rm, H.rowmap); PUT(wo, H.woff); PUT(pm, H.pmap); PUT(pi, H.pidx); PUT(ws, H.wsplit);
        G.rowmap = rm; G.woff = wo; G.pmap = pm; G.pidx = pi; G.wsplit = ws;
        if (H.tile && (G.merged || G.sd)) { G.pj = nullptr; G.pj32 = nullptr; }   // the fused product reads J once
        else if (fp32_jac) { ALLOC(G.pj32, 3 * 64 * G.nslots); }
        else { ALLOC(G.pj, 3 * 64 * G.nslots); }
        H.pmap.clear(); H.pmap.shrink_to_fit();
        H.pidx.clear(); H.pidx.shrink_to_fit();
    }
    ALLOC(G.Hv, 6 * (int64_t)nown); ALLOC(G.Dv, 6 * (int64_t)nown); ALLOC(G.Mv, 6 * (int64_t)nown);
    ALLOC(G.cdep, 3 * (int64_t)nd); ALLOC(G.wss, nd);
    ALLOC(G.hl, 21 * (int64_t)Q + S + G.ndof);
    G.b = G.hl + 21 * (int64_t)Q + S;
    ALLOC(G.Mh, 36 * (int64_t)Q + S);
    ALLOC(G.lpart, (int64_t)kSpLin * G.nblk); ALLOC(G.mpart, std::max(std::max(G.nrb2, 8 * ((G.nrb + 7) / 8)), 1));
    ALLOC(G.r, G.ndof); ALLOC(G.q, G.ndof); ALLOC(G.x, G.ndof);
    // zp: [heavy][rows][receive region: the halo rows, 3 dofs each, in the concatenated receive order]
    int64_t nrecv = 0;
    for (const auto &v : H.recv_rows) nrecv += (int64_t)v.size();
    const int64_t zp_n = G.ndof + (G.sd ? 3 * nrecv : 0);
    double *zp;
    ALLOC(zp, 2 * zp_n);
    G.zp = reinterpret_cast<double2 *>(zp);
    if (H.tile && (G.merged || G.sd)) {
        G.tile = 1;
        G.ntile = H.ntile;
        G.tile_lds = H.tile_lds;
        G.tile_segmax = H.tile_segmax;
        G.t_grid = 8 * ((H.ntile + 7) / 8) + 1;
        int32_t *tt, *trs, *th, *txo, *txd, *tch;
        uint32_t *tm;
        // halo rows as zp rows: this rank's (global row = row0 + local) as they are, another rank's
        // at NP + its position in the concatenated receive lists (ascending: the peers' ranges ascend)
        std::vector<int32_t> hz(H.tile_halo);
        if (nranks_ > 1) {
            std::vector<int32_t> rr;
            for (const auto &v : H.recv_rows) rr.insert(rr.end(), v.begin(), v.end());
            for (auto &r : hz)
                if (r < H.lo || r >= H.hi) {
                    const auto itr = std::lower_bound(rr.begin(), rr.end(), r);
                    if (itr == rr.end() || *itr != r) return fail(DEFTRI_E_ARG, "tile plan: a halo row is neither own nor received");
                    r = NP + (int32_t)(itr - rr.begin());
                }
        }
        PUT(tt, H.tile_tab); PUT(trs, H.tile_rs); PUT(th, hz); PUT(txo, H.tile_xoff); PUT(txd, H.tile_xdst);
        PUT(tch, H.tile_chunk);
        {
            std::vector<uint32_t> mm(2 * H.tile_m0.size());
            for (size_t k = 0; k < H.tile_m0.size(); k++) { mm[2 * k] = H.tile_m0[k]; mm[2 * k + 1] = H.tile_m1[k]; }
            PUT(tm, mm);
        }
        G.ttab = tt; G.trs = trs; G.thalo = th; G.txoff = txo;
        if (H.tile_multi) {                        // several pairs: own-row lists, shares, pair ranges
            int32_t *tr, *tdd, *tpo, *tns, *tdp;
            PUT(tr, H.tile_trow); PUT(tdd, H.tile_tdst); PUT(tpo, H.tile_poff); PUT(tns, H.tile_nshare);
            // each tile row's depth edge in the tile's pair (the reference gives a point one depth edge
            // per pair, on the scale of its keyframe in that pair): 2 j + (scale & 1), or -1
            std::vector<int32_t> tdep(H.tile_trow.size(), -1);
            std::atomic<int> twice{0};
            chunked(H.ntile, 256, [&](int, int64_t t0, int64_t t1) {
                for (int64_t t = t0; t < t1; t++) {
                    const int32_t *T = &H.tile_tab[8 * (size_t)t];
                    for (int32_t i = 0; i < T[1]; i++) {
                        const int32_t l = H.tile_trow[T[0] + i] & 0x7fffffff;
                        for (int32_t j = H.dep_off[l]; j < H.dep_off[l + 1]; j++) {
                            if ((ds[j] >> 1) != T[7]) continue;
                            if (tdep[T[0] + i] >= 0 || j >= (1 << 30)) twice = 1;
                            tdep[T[0] + i] = 2 * j + (ds[j] & 1);
                        }
                    }
                }
            });
            if (twice) return fail(DEFTRI_E_ARG, "tile plan: a row with two depth edges in one pair");
            PUT(tdp, tdep);
            G.tmulti = 1;
            G.trow = tr; G.tdst = tdd; G.tpoff = tpo; G.tnshare = tns; G.tdep = tdp;
            ALLOC(G.qs, 3 * std::max<int64_t>((int64_t)H.tile_planes * nown, 1));
        }
        G.txdst = reinterpret_cast<const int2 *>(txd);
        G.tchunk = reinterpret_cast<const int2 *>(tch);
        G.tmeta = reinterpret_cast<const uint2 *>(tm);
        G.pinfo = P.pair_info;
        ALLOC(G.xc, 3 * std::max<int64_t>(H.tile_cross, 1));    // 3 per cross slot
        // each product launch sums the last update's (r.z, r.r) partials itself, and each update
        // workgroup alpha from the product's; only the chain's last update takes the ticketed sum that
        // records the state.  Every workgroup reading every partial costs O(workgroups^2) reads, so
        // from kSpTilePartsMax tiles (the multi-keyframe graphs: C3 has 12k) the ticketed sums and the
        // alpha hand-off take over, as on the sharded chain (whose record is all-reduced)
        G.tparts = (G.sd || G.t_grid > kSpTilePartsMax) ? 0 : 1;
        // sharded: the rank's record xb in its own small launch (k_sp_txb) — forming it in the
        // product's last workgroup instead (a ticket over both product launches) measured the same on
        // the 2-rank gloo rehearsal (165.8 vs 171.8 LM it/s), so the simpler order stays
    }
    ALLOC(G.s, nloc); ALLOC(G.part, (int64_t)kSpPart * std::max(G.nblk, G.t_grid)); ALLOC(G.rpart, std::max(G.nrb2, 1));
    ALLOC(G.upart, 2 * (int64_t)(G.nrb + 1)); ALLOC(G.hbuf, 1 + H.hd);
    ALLOC(G.rec, kSpRecDoubles + (int64_t)kSpRed * (kSpMaxIt + 2));
    ALLOC(G.ph, std::max<int64_t>(H.hd, 1));
    G.m1n = G.tile ? G.t_grid : sp_merged_grid1(G);
    ALLOC(G.m1part, std::max(G.m1n, sp_merged_grid1(G)));
    ALLOC(G.m2part, 2 * (int64_t)std::max(sp_merged_grid2(G), G.m_nh + 8 * ((G.nrb + 7) / 8))); ALLOC(G.gsum, 32);
    ALLOC(G.cnt, 64);      // three ticket sites (0, 16, 32: 9 counters each), the tile arrival (44), the sharded tiles' (48)
    SPOK(hipMemset(G.cnt, 0, 64 * sizeof(int)));
    {
        // heavy linearization chunks (k_sp_glin_heavy): kSpHeavyChunk block partials each, >= 1 per vertex
        std::vector<int32_t> chh, hcho(Q + S + 1, 0);
        std::vector<int64_t> chlo;
        for (int32_t h = 0; h < Q + S; h++) {
            const int64_t k0 = H.hv_blk_off[h], k1 = H.hv_blk_off[h + 1];
            int64_t k = k0;
            do {
                chh.push_back(h);
                chlo.push_back(k);
                k = std::min<int64_t>(k + kSpHeavyChunk, k1);
            } while (k < k1);
            hcho[h + 1] = (int32_t)chh.size();
        }
        chlo.push_back(H.hv_blk_off.empty() ? 0 : H.hv_blk_off.back());
        G.nch = (int32_t)chh.size();
        int32_t *d_chh, *d_hcho;
        int64_t *d_chlo;
        PUT(d_chh, chh); PUT(d_hcho, hcho); PUT(d_chlo, chlo);
        G.ch_h = d_chh; G.hch_off = d_hcho; G.ch_lo = d_chlo;
        ALLOC(G.chpart, (int64_t)kSpLin * std::max(G.nch, 1));
        ALLOC(G.hcnt, std::max(Q + S, 1));
        SPOK(hipMemset(G.hcnt, 0, sizeof(int) * (size_t)std::max(Q + S, 1)));
    }
    G.red = G.rec + kSpRecDoubles;
    SPOK(hipMemset(G.x, 0, sizeof(double) * (size_t)G.ndof));     // rows no solve writes stay 0
    SPOK(hipMemset(G.zp, 0, sizeof(double) * 2 * (size_t)zp_n));
    SPOK(hipMemset(G.rec, 0, sizeof(double) * (size_t)(kSpRecDoubles + kSpRed * (kSpMaxIt + 2))));
    ALLOC(d_scal, 8); ALLOC(d_part, kMaxSumJobs * kSpRedParts); ALLOC(d_flag, 1); ALLOC(d_sumcnt, 16);
    {                                  // the trial evaluation's partials: every edge kind and the whole dx
        EvalJob ej;
        ej.n_arap = H.n_arap_owned;
        ej.n_den = G.ndof;
        n_epart_ = trial_eval_parts(P, ej);
        ALLOC(d_epart, n_epart_);
        if (h_epart_) hipHostFree(h_epart_);
        h_epart_ = nullptr;
        SPOK(hipHostMalloc((void **)&h_epart_, sizeof(double) * (size_t)n_epart_, hipHostMallocDefault));
        // the linearization's chi2 partials (one rank; sharded contexts keep the per-edge chi2 sums)
        P.n_arap_sum = H.n_arap_owned;
        lin_chi_blocks(P, lin_nb_);
        const int64_t nl = std::max<int64_t>(1, (int64_t)lin_nb_[0] + lin_nb_[1] + lin_nb_[2]);
        ALLOC(d_lpart_, nl);
        if (h_lpart_) hipHostFree(h_lpart_);
        h_lpart_ = nullptr;
        SPOK(hipHostMalloc((void **)&h_lpart_, sizeof(double) * (size_t)nl, hipHostMallocDefault));
    }
    SPOK(hipMemset(d_flag, 0, sizeof(int)));
    SPOK(hipMemset(d_sumcnt, 0, 16 * sizeof(int)));
    ALLOC(d_tmp, G.ndof); ALLOC(d_dx0, G.ndof);
    PUT(d_row_of_point, H.row_of_point);
    // halo lists: per peer, sends then receives, 6 doubles per row ((z, p) of 3 dofs)
    std::vector<int32_t> srows, rrows;
    send_off_.assign(nranks_ + 1, 0);
    recv_off_.assign(nranks_ + 1, 0);
    for (int p = 0; p < nranks_; p++) {
        srows.insert(srows.end(), H.send_rows[p].begin(), H.send_rows[p].end());
        rrows.insert(rrows.end(), H.recv_rows[p].begin(), H.recv_rows[p].end());
        send_off_[p + 1] = (int64_t)srows.size();
        recv_off_[p + 1] = (int64_t)rrows.size();
    }
    PUT(d_send_rows, srows); PUT(d_recv_rows, rrows);
    ALLOC(d_xbuf, 6 * (int64_t)(srows.size() + rrows.size()));
    if (G.sd) {
        ALLOC(G.sv, G.ndof);
        SPOK(hipMemset(G.sv, 0, sizeof(double) * (size_t)G.ndof));
        ALLOC(G.xb, 3 + H.hd);
        G.sbuf = d_xbuf;                                   // the send half of the halo buffer
        // phase 1's rows: a halo row (recv list position k, concatenated in peer order — the peers'
        // row ranges ascend, so the concatenation is sorted) reads its (z, p) at row P + k
        std::vector<int32_t> ap(4 * (size_t)nloc);
        for (int64_t le = 0; le < nloc; le++)
            for (int k = 0; k < 4; k++) {
                const int32_t r = H.row_of_point[d.arap_pts[4 * H.arap_ids[le] + k]];
                int32_t m = r;
                if (r < H.lo || r >= H.hi) {
                    const auto it = std::lower_bound(rrows.begin(), rrows.end(), r);
                    if (it == rrows.end() || *it != r) return fail(DEFTRI_E_ARG, "iterative plan: a local edge's row is neither own nor halo");
                    m = NP + (int32_t)(it - rrows.begin());
                }
                ap[4 * le + k] = m;
            }
        int32_t *d_ap;
        PUT(d_ap, ap);
        G.apts_p = d_ap;
        // own row l -> its send slots (rows of sbuf), in the concatenated send order
        std::vector<int32_t> so(nown + 1, 0), sl;
        for (int32_t r : srows) so[r - H.lo + 1]++;
        for (int32_t l = 0; l < nown; l++) so[l + 1] += so[l];
        sl.resize(srows.size());
        std::vector<int32_t> fill(so.begin(), so.end() - 1);
        for (size_t k = 0; k < srows.size(); k++) sl[fill[srows[k] - H.lo]++] = (int32_t)k;
        int32_t *d_so, *d_sl;
        PUT(d_so, so); PUT(d_sl, sl);
        G.snd_off = d_so; G.snd_slot = d_sl;
        // the halo exchange beside phase 1's interior workgroups: phase-1 blocks whose
        // ARAP edges read no halo row (and the heavy / row-term workgroups) run while the boundary
        // rows' (z, p) travel; the blocks that read one wait for them.  DEFTRI_SP_NO_OVERLAP=1: one
        // phase-1 launch after the exchange (round 4)
        static const bool no_ovl = std::getenv("DEFTRI_SP_NO_OVERLAP") != nullptr;
        G.ovl = (nranks_ > 1 && !no_ovl) ? 1 : 0;
        if (G.ovl && G.tile) {
            // the tile chain: the workgroups of tiles that read no other rank's row (and the heavy
            // one, and the empty slots) beside the exchange, the others after it
            std::vector<int32_t> li, lb;
            const int32_t seg = (H.ntile + 7) / 8;
            for (int32_t b = 0; b < G.t_grid; b++) {
                const int32_t t = b == G.t_grid - 1 ? H.ntile : (b & 7) * seg + (b >> 3);
                bool bnd = false;
                if (t < H.ntile) {
                    const int32_t *T = &H.tile_tab[8 * (size_t)t];
                    for (int32_t k = T[5]; k < T[5] + T[2] && !bnd; k++) bnd = H.tile_halo[k] < H.lo || H.tile_halo[k] >= H.hi;
                }
                (bnd ? lb : li).push_back(b);
            }
            n_p1int = (int)li.size();
            n_p1bnd = (int)lb.size();
            PUT(d_p1int, li);
            if (lb.empty()) lb.push_back(0);
            PUT(d_p1bnd, lb);
            if (!cs_) SPOK(hipStreamCreateWithFlags(&cs_, hipStreamNonBlocking));
            if (!ev_upd_) SPOK(hipEventCreateWithFlags(&ev_upd_, hipEventDisableTiming));
            if (!ev_halo_) SPOK(hipEventCreateWithFlags(&ev_halo_, hipEventDisableTiming));
        } else if (G.ovl) {
            std::vector<int32_t> li, lb;
            for (int32_t e = 0; e < G.m_nx; e++) li.push_back(e);
            for (int32_t b = 0; b < G.nblk; b++) {
                const int32_t *d4 = &H.blk[4 * (size_t)b];
                bool bnd = false;
                if ((d4[0] & 0xff) == SP_ARAP)
                    for (int32_t le = d4[2]; le < d4[3] && !bnd; le++)
                        for (int k = 0; k < 4; k++) bnd |= ap[4 * (size_t)le + k] >= NP;
                (bnd ? lb : li).push_back(G.m_nx + b);
            }
            n_p1int = (int)li.size();
            n_p1bnd = (int)lb.size();
            PUT(d_p1int, li);
            if (lb.empty()) lb.push_back(0);
            PUT(d_p1bnd, lb);
            if (!cs_) SPOK(hipStreamCreateWithFlags(&cs_, hipStreamNonBlocking));
            if (!ev_upd_) SPOK(hipEventCreateWithFlags(&ev_upd_, hipEventDisableTiming));
            if (!ev_halo_) SPOK(hipEventCreateWithFlags(&ev_halo_, hipEventDisableTiming));
        }
        int_pending_ = -1;
    } else {
        G.apts_p = G.apts;
    }
#undef PUT
#undef ALLOC
    SPOK(hipDeviceSynchronize());
    have_ = true;
    return 0;
}

// halo exchange of the boundary rows: zp (6 doubles per row: (z, p) of its 3 dofs) or x (3)
int SpSolver::halo(int width, double *vec, bool zp) {
    if (nranks_ <= 1) return 0;
    const int64_t base = zp ? 2 * G.hd : G.hd;
    const int64_t nsend = send_off_[nranks_];
    double *sbuf = d_xbuf, *rbuf = d_xbuf + 6 * nsend;
    sp_launch_halo_pack((int)nsend, d_send_rows, width, base, vec, sbuf, st_);
    // global order: for every (src, dst) pair in lexicographic order, the src sends and the dst receives
    std::vector<SpTransport::Op> ops;
    for (int a = 0; a < nranks_; a++)
        for (int b = 0; b < nranks_; b++) {
            if (a == b) continue;
            if (a == rank_ && send_off_[b + 1] > send_off_[b])
                ops.push_back({b, true, sbuf + width * send_off_[b], width * (send_off_[b + 1] - send_off_[b])});
            if (b == rank_ && recv_off_[a + 1] > recv_off_[a])
                ops.push_back({a, false, rbuf + width * recv_off_[a], width * (recv_off_[a + 1] - recv_off_[a])});
        }
    int rc = tr_->p2p(ops, st_);
    if (rc) return rc;
    sp_launch_halo_unpack((int)recv_off_[nranks_], d_recv_rows, width, base, rbuf, vec, st_);
    return 0;
}

// the sd chain's halo exchange: the boundary rows' (z, p) from the send buffer k_sp_update_sd (or
// the setup) filled straight into the peers' receive regions of zp
int SpSolver::halo_sd() {
    if (!shard_ || nranks_ <= 1) return 0;
    if (G.ovl) SPOK(hipStreamWaitEvent(cs_, ev_upd_, 0));    // (the send buffer written on st_)
    const int64_t nsend = send_off_[nranks_];
    double *sbuf = G.sbuf, *rbuf = reinterpret_cast<double *>(G.zp + G.ndof);
    std::vector<SpTransport::Op> ops;
    for (int a = 0; a < nranks_; a++)
        for (int b = 0; b < nranks_; b++) {
            if (a == b) continue;
            if (a == rank_ && send_off_[b + 1] > send_off_[b])
                ops.push_back({b, true, sbuf + 6 * send_off_[b], 6 * (send_off_[b + 1] - send_off_[b])});
            if (b == rank_ && recv_off_[a + 1] > recv_off_[a])
                ops.push_back({a, false, rbuf + 6 * recv_off_[a], 6 * (recv_off_[a + 1] - recv_off_[a])});
        }
    (void)nsend;
    if (!G.ovl) return tr_->p2p(ops, st_);
    const int rc = tr_->p2p(ops, cs_);
    if (rc) return rc;
    SPOK(hipEventRecord(ev_halo_, cs_));
    return 0;
}

// the sharded chain's product of iteration it: phase 1 (G.ovl: the interior workgroups unless
// already queued, the wait for the exchange, the boundary ones), phase 2
int SpSolver::sd_product(int it, double lambda) {
    const bool f32 = fp32_jac != 0;
    if (G.tile) {                                  // w = A z by tiles, the rank's record xb
        if (!G.ovl) {
            sp_launch_tile_sd(G, it, lambda, f32, st_, nullptr, G.t_grid, true);
            return 0;
        }
        if (int_pending_ != it) sp_launch_tile_sd(G, it, lambda, f32, st_, d_p1int, n_p1int, false);
        int_pending_ = -1;
        SPOK(hipStreamWaitEvent(st_, ev_halo_, 0));
        sp_launch_tile_sd(G, it, lambda, f32, st_, d_p1bnd, n_p1bnd, true);
        return 0;
    }
    if (!G.ovl) {
        sp_launch_sd_phase1(G, it, lambda, f32, st_, nullptr, sp_merged_grid1(G));
    } else {
        if (int_pending_ != it) sp_launch_sd_phase1(G, it, lambda, f32, st_, d_p1int, n_p1int);
        int_pending_ = -1;
        SPOK(hipStreamWaitEvent(st_, ev_halo_, 0));
        sp_launch_sd_phase1(G, it, lambda, f32, st_, d_p1bnd, n_p1bnd);
    }
    sp_launch_sd_phase2(G, it, lambda, f32, st_);
    return 0;
}

// after the update (or the setup) wrote the boundary rows' (z, p): G.ovl — queue iteration next_it's
// interior phase 1, then the exchange on cs_ beside it (a host transport blocks this thread while
// the device runs it); otherwise the exchange on st_
int SpSolver::sd_exchange(int next_it, double lambda) {
    if (!G.ovl) return halo_sd();
    SPOK(hipEventRecord(ev_upd_, st_));
    if (G.tile) sp_launch_tile_sd(G, next_it, lambda, fp32_jac != 0, st_, d_p1int, n_p1int, false);
    else sp_launch_sd_phase1(G, next_it, lambda, fp32_jac != 0, st_, d_p1int, n_p1int);
    int_pending_ = next_it;
    return halo_sd();
}

// computeActiveErrors (+ linearizeOplus with jac) on the rank's edges, chi2 of its owned edges into
// d_scal[slot]; `extra`: one more fixed-order sum in the same launches (the rho denominator)
int SpSolver::eval_chi2(bool analytic, int slot, const SumJob *extra, const ReadBack *rb, double *h_part,
                        double *rec_clear, int64_t nclear) {
    (void)analytic;                  // errors only: the Jacobian mode does not enter
    // the edges' errors and every sum in one launch (k_trial_eval)
    EvalJob J;
    J.n_arap = H.n_arap_owned;
    J.out = d_scal + 4;
    if (extra) {
        if (extra->mode != 1) return fail(DEFTRI_E_ARG, "trial evaluation: the extra sum must be dx.(lambda dx + b)");
        J.dx = extra->a; J.b = extra->b; J.n_den = extra->n;
        J.lambda = extra->lambda; J.lambda_dev = extra->lambda_dev; J.den_out = extra->out;
    }
    J.total = d_scal + slot;
    J.gate = P.gate_trial;
    J.h_part = h_part;
    if (h_part && rec_clear) { J.rec_clear = rec_clear; J.nclear = nclear; J.flag_clear = d_flag; }
    trial_eval_blocks(P, J, eval_nb_);
    if (trial_eval_parts(P, J) > n_epart_) return fail(DEFTRI_E_ARG, "trial evaluation: partial buffer too small");
    launch_trial_eval(P, J, d_epart, d_sumcnt, rb ? *rb : ReadBack{}, st_);
    return 0;
}

// per LM iteration: linearize, chi2 (reduced), the rows' / heavy blocks and b (heavy reduced), and at
// iteration 0 max diag H into d_scal[2]
double SpSolver::lin_chi_host() const {
    double s4[4];
    trial_eval_host_sums(h_lpart_, lin_nb_, s4);
    return (s4[0] + s4[2]) + s4[1];
}

// host_chi (one rank, the host loop): the chi2 partials go to pinned memory and the caller adds them
// (lin_chi_host) after its next synchronization; d_scal[0] is then not written
int SpSolver::lin_iteration(bool analytic, bool want_max, bool &ok, bool host_chi) {
    ok = true;
    lin_host_pending_ = false;
    if (!shard_) {
        // per-workgroup chi2 partials from the linearization's own launches (no per-edge chi2, no
        // separate sum launch on the host loop)
        P.lin_part = host_chi ? h_lpart_ : d_lpart_;
        launch_linearize(P, st_, true, analytic);
        P.lin_part = nullptr;
        if (host_chi) lin_host_pending_ = true;
        else launch_part_sums(d_lpart_, lin_nb_, d_scal + 4, nullptr, d_scal, P.gate_lin, st_);
    } else {
        launch_linearize(P, st_, true, analytic);
        SumJobs J;
        J.j[0].n = P.R; J.j[0].a = P.chi_rep; J.j[0].out = d_scal + 4;
        J.j[1].n = P.D; J.j[1].a = P.chi_dep; J.j[1].out = d_scal + 5;
        J.j[2].n = H.n_arap_owned; J.j[2].a = P.chi_arap; J.j[2].out = d_scal + 6;
        J.nj = 3;
        J.total = d_scal;
        launch_sum_multi_fused(J, d_part, kSumParts, d_sumcnt, ReadBack{}, st_);
    }
    int rc;
    if (shard_ && (rc = tr_->allreduce(d_scal, 1, 0, st_))) return rc;
    if (fp32_jac) sp_launch_cvt_j(P.Jarap, const_cast<float *>(G.Ja32), 18 * G.jld, st_);
    sp_launch_glin(G, fp32_jac != 0, st_);
    if (shard_ && (rc = tr_->allreduce(G.hl, 21 * (int64_t)G.Q + G.S + G.hd, 0, st_))) return rc;
    if (want_max) {
        sp_launch_maxdiag(G, d_scal + 2, st_);
        if (shard_ && (rc = tr_->allreduce(d_scal + 2, 1, 1, st_))) return rc;
        sp_launch_maxdiag_heavy(G, d_scal + 2, st_);
    }
    return 0;
}

// the solve's setup (preconditioner at lambda, r = rhs, (z, p) = (M r, 0), x = 0); sharded: the
// boundary rows' (z, p) to the ranks whose edges read them, as after every CG update
int SpSolver::cg_setup(double lambda, const double *rhs) {
    if (G.ovl) SPOK(hipStreamWaitEvent(st_, ev_halo_, 0));   // (no exchange of an earlier solve in flight)
    int_pending_ = -1;
    sp_launch_setup(G, rhs, lambda, st_);
    if (G.sd) return sd_exchange(0, lambda);
    if (shard_) return halo(6, reinterpret_cast<double *>(G.zp), true);
    return 0;
}

// CG iterations [from, to) at lambda; every transport call's status is checked (a failed collective
// must not leave the ranks iterating on stale data)
int SpSolver::cg_chain(double lambda, int from, int to) {
    int rc;
    for (int it = from; it < to; it++) {
        if (G.sd) {                                    // phase 1, phase 2 (A z), one all-reduce, update
            if ((rc = sd_product(it, lambda))) return rc;
            if ((rc = tr_->allreduce(G.xb, 3 + G.hd, 0, st_))) return rc;
            sp_launch_update_sd(G, it, lambda, 0, st_);
            if ((rc = sd_exchange(it + 1, lambda))) return rc;
            continue;
        }
        if (G.merged) {                                // phase 1 (+ alpha), phase 2 (+ update, next dots)
            sp_launch_product(G, it, lambda, fp32_jac != 0, st_, it == to - 1);
            continue;
        }
        const bool dist = shard_;
        if (!G.fuse) sp_launch_dots(G, it, st_);      // fused: the previous update's (setup's) last workgroup
        if (dist && (rc = tr_->allreduce(G.red + (int64_t)kSpRed * it, 2, 0, st_))) return rc;
        sp_launch_product(G, it, lambda, fp32_jac != 0, st_);
        if (dist) {
            sp_launch_heavy(G, it, lambda, 1, st_);
            if ((rc = tr_->allreduce(G.hbuf, 1 + G.hd, 0, st_))) return rc;
            sp_launch_heavy(G, it, lambda, 2, st_);
        } else if (G.fuse_heavy) {
            // in k_sp_phase2's last workgroup
        } else if (G.heavy_split) {
            sp_launch_heavy(G, it, lambda, 1, st_);
            sp_launch_heavy(G, it, lambda, 2, st_);
        } else {
            sp_launch_heavy(G, it, lambda, 0, st_);
        }
        sp_launch_update(G, it, st_);
        if (dist && (rc = halo(6, reinterpret_cast<double *>(G.zp), true))) return rc;
    }
    return 0;
}

// the state of iteration n into the record (converged / budget), no other effect (the sd chain
// decides it after iteration n's product and reduction: they run, the update records only)
int SpSolver::cg_tail(int n, double lambda) {
    int rc;
    if (G.merged) return 0;                            // phase 2's last workgroup records iteration n's state
    if (G.sd) {
        if ((rc = sd_product(n, lambda))) return rc;
        if ((rc = tr_->allreduce(G.xb, 3 + G.hd, 0, st_))) return rc;
        sp_launch_update_sd(G, n, lambda, 1, st_);
        return 0;
    }
    if (!G.fuse) sp_launch_dots(G, n, st_);
    if (shard_ && (rc = tr_->allreduce(G.red + (int64_t)kSpRed * n, 2, 0, st_))) return rc;
    // k_sp_heavy stage 1 records the state of a finished solve and returns; a running one would
    // compute its sums, so the tail records through stage 1 only when the state is final: launch
    // the status-only variant (stage 3)
    sp_launch_heavy(G, n, 0.0, 3, st_);
    return 0;
}

// one step (H + lambda I) x = rhs into G.x with polling (diagnostics / profiling path)
int SpSolver::pcg_solve(double lambda, const double *rhs, bool &solved, int &its) {
    const int mx = budget();
    G.max_it = mx;
    G.tol2 = tol * tol;
    SPOK(hipMemsetAsync(G.rec, 0, sizeof(double) * (size_t)(kSpRecDoubles + kSpRed * (mx + 2)), st_));
    int rc = cg_setup(lambda, rhs);
    if (rc) return rc;
    int j = 0;
    int n = std::min(std::max(2, last_its + 1), mx);
    for (;;) {
        if ((rc = cg_chain(lambda, j, n))) return rc;
        j = n;
        if ((rc = cg_tail(j, lambda))) return rc;
        SPOK(hipMemcpyAsync(hpin + 16, G.rec, sizeof(double) * kSpRecDoubles, hipMemcpyDeviceToHost, st_));
        SPOK(hipStreamSynchronize(st_));
        const int status = (int)hpin[16];
        if (status == kSpTimeout) return hand_off_timeout();
        if (status == kSpConverged) { its = (int)hpin[17]; solved = true; break; }
        if (status != kSpRunning || j >= mx) { its = j; solved = false; break; }
        n = std::min(j + 4, mx);
    }
    if (solved) last_its = its;
    step_its = its;
    step_solved = solved ? 1 : 0;
    return 0;
}

// ---- device-driven LM (one rank) ------------------------------------------------------------------
// The LM's decisions (rho, accept / reject, lambda and nu, g2o's loop and Terminate conditions) run on
// the device (kernels.hip k_lm_decide), so the host queues "slots" — [linearization, gated on the
// last trial's acceptance] [prologue: backup or restore] [setup, CG chain, tail, evaluation] [decide]
// — without waiting for each trial's outcome.  It keeps two slots in flight and reads the decision of
// the oldest one (an event per slot; the decide kernel copies the state to pinned memory); a slot
// queued past the end of the solve returns at once in every kernel.  A step whose PCG needs more
// iterations than its slot queued (the host's guess: the last converged count + 2) stops the slots
// (stop 3): the host continues that solve in chunks of 4 exactly as solve_lm's host loop does, then
// queues the evaluation and the decide.  Identical arithmetic and decisions as the host loop
// (tests/test_gpu_sp.py::test_device_lm_matches_host_lm).  Opt-in: DEFTRI_DEVICE_LM=1.
int SpSolver::solve_lm_dev(const deftri_lm_params &prm, deftri_report &R) {
    hipSetDevice(dev_);
    auto t_start = std::chrono::steady_clock::now();
    const int max_trials = prm.max_trials > 0 ? prm.max_trials : 10;
    const double tau = prm.tau > 0 ? prm.tau : 1e-5;
    const bool analytic = prm.analytic_jacobians != 0;
    const int mx = budget();
    const int64_t nrec = kSpRecDoubles + (int64_t)kSpRed * (mx + 2);
    int rc;
    if (!d_lm) {
        if ((rc = alloc(&d_lm, 1)) || (rc = alloc(&d_chi_it, DEFTRI_MAX_REPORT_ITERS)) ||
            (rc = alloc(&d_trials_it, DEFTRI_MAX_REPORT_ITERS)))
            return rc;
        SPOK(hipHostMalloc((void **)&h_snap, sizeof(LmState), hipHostMallocDefault));
    }
    if ((rc = save_entry())) return rc;
    eval_chi2(analytic, 0, nullptr);
    SPOK(hipMemcpyAsync(hpin, d_scal, sizeof(double), hipMemcpyDeviceToHost, st_));
    SPOK(hipStreamSynchronize(st_));
    R.chi2_initial = hpin[0];
    LmState L{};
    L.lam = 0.0; L.ni = 2.0; L.cur = R.chi2_initial;
    L.gate_trial = prm.n_iterations > 0 ? 1 : 0;
    L.gate_lin = L.gate_trial;
    L.need_lin = 1;
    L.stop = prm.n_iterations > 0 ? 0 : 1;
    L.last_its = last_its;
    L.n_it = prm.n_iterations;
    L.max_trials = max_trials;
    L.slot = L.stop_slot = -1;
    *h_snap = L;
    SPOK(hipMemcpyAsync(d_lm, &L, sizeof(LmState), hipMemcpyHostToDevice, st_));
    SPOK(hipMemsetAsync(d_trials_it, 0, sizeof(int32_t) * DEFTRI_MAX_REPORT_ITERS, st_));
    // gates and lambda from the state
    P.gate_lin = &d_lm->gate_lin;
    P.gate_trial = &d_lm->gate_trial;
    G.gate = &d_lm->gate_trial;
    G.lgate = &d_lm->gate_lin;
    G.lam_dev = &d_lm->lam;
    G.max_it = mx;
    G.tol2 = tol * tol;
    struct Clear {              // the gates off again whatever path leaves this function
        SpSolver *s;
        ~Clear() { s->P.gate_lin = s->P.gate_trial = nullptr; s->G.gate = s->G.lgate = nullptr; s->G.lam_dev = nullptr; }
    } clear{this};
    // the evaluation of a slot's step: state update, chi2 + the rho denominator (lambda from HBM)
    auto evaluate = [&]() {
        launch_update_state(P, G.x, st_, nullptr);
        SumJob den;
        den.n = G.hd + 3 * (int64_t)G.nown; den.a = G.x; den.b = G.b; den.lambda_dev = &d_lm->lam;
        den.mode = 1; den.out = d_scal + 1;
        return eval_chi2(analytic, 0, &den);     // gated by P.gate_trial (= the LM state's gate_trial)
    };
    struct Slot { int idx, n; hipEvent_t ev; };
    std::vector<hipEvent_t> evpool;
    std::vector<Slot> inflight;
    int queued = 0, guess = std::max(2, last_its + 2);
    auto enqueue = [&]() -> int {
        const bool first = queued == 0;
        // linearization (gate_lin): errors + Jacobians, chi2 sums, the rows' / heavy blocks, b
        // (the host loop's partials and order: bit-identical chi2)
        P.lin_part = d_lpart_;
        launch_linearize(P, st_, true, analytic);
        P.lin_part = nullptr;
        launch_part_sums(d_lpart_, lin_nb_, d_scal + 4, nullptr, d_scal, &d_lm->gate_lin, st_);
        if (fp32_jac) sp_launch_cvt_j(P.Jarap, const_cast<float *>(G.Ja32), 18 * G.jld, st_, &d_lm->gate_lin);
        sp_launch_glin(G, fp32_jac != 0, st_);
        if (first) {
            sp_launch_maxdiag(G, d_scal + 2, st_);
            sp_launch_maxdiag_heavy(G, d_scal + 2, st_);
        }
        // the trial (gate_trial)
        launch_trial_begin_dev(P, d_flag, G.rec, nrec, d_lm, d_scal, tau, prm.user_lambda, st_);
        int r2;
        if ((r2 = cg_setup(0.0, G.b))) return r2;
        const int n = std::min(guess, mx);
        if ((r2 = cg_chain(0.0, 0, n))) return r2;
        if ((r2 = cg_tail(n, 0.0))) return r2;
        if ((r2 = evaluate())) return r2;
        launch_lm_decide(d_lm, d_scal, G.rec, d_chi_it, d_trials_it, DEFTRI_MAX_REPORT_ITERS, h_snap, queued, st_);
        if (evpool.empty()) { hipEvent_t e; SPOK(hipEventCreateWithFlags(&e, hipEventDisableTiming)); evpool.push_back(e); }
        hipEvent_t e = evpool.back();
        evpool.pop_back();
        SPOK(hipEventRecord(e, st_));
        inflight.push_back({queued, n, e});
        queued++;
        return 0;
    };
    std::vector<int> slot_n;            // CG iterations queued per enqueue index
    bool host_stop = false;
    for (;;) {
        while (!host_stop && inflight.size() < 2) {
            if ((rc = enqueue())) return rc;
            slot_n.push_back(inflight.back().n);
        }
        if (inflight.empty()) break;
        const Slot sl = inflight.front();
        inflight.erase(inflight.begin());
        SPOK(hipEventSynchronize(sl.ev));
        evpool.push_back(sl.ev);
        const LmState S = *h_snap;
        if (S.last_its > 0) guess = std::max(2, S.last_its + 2);
        if (S.stop == 4) {                                 // alpha hand-off timeout: an error, not a trial
            SPOK(hipStreamSynchronize(st_));
            for (const Slot &o : inflight) evpool.push_back(o.ev);
            for (hipEvent_t e : evpool) hipEventDestroy(e);
            return hand_off_timeout();
        }
        if (S.stop == 1 || S.stop == 2) { host_stop = true; continue; }
        if (S.stop == 3) {
            // the slot S.stop_slot queued too few CG iterations: every later slot returned at once
            SPOK(hipStreamSynchronize(st_));
            for (const Slot &o : inflight) evpool.push_back(o.ev);
            inflight.clear();
            int j = slot_n[S.stop_slot];
            // the evaluation applied the unfinished x: restore, continue the solve in chunks of 4
            SPOK(hipMemcpyAsync(P.points, P.points_bak, sizeof(double) * 3 * (size_t)P.P, hipMemcpyDeviceToDevice, st_));
            SPOK(hipMemcpyAsync(P.scales, P.scales_bak, sizeof(double) * (size_t)P.S, hipMemcpyDeviceToDevice, st_));
            SPOK(hipMemcpyAsync(P.tg, P.tg_bak, sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToDevice, st_));
            const int one = 1, zero = 0;
            SPOK(hipMemcpyAsync(&d_lm->gate_trial, &one, sizeof(int), hipMemcpyHostToDevice, st_));
            SPOK(hipMemcpyAsync(&d_lm->stop, &zero, sizeof(int), hipMemcpyHostToDevice, st_));
            int st = kSpRunning;
            while (st == kSpRunning && j < mx) {
                const int n2 = std::min(j + 4, mx);
                if ((rc = cg_chain(0.0, j, n2))) return rc;
                j = n2;
                if ((rc = cg_tail(j, 0.0))) return rc;
                SPOK(hipMemcpyAsync(hpin + 16, G.rec, sizeof(double) * kSpRecDoubles, hipMemcpyDeviceToHost, st_));
                SPOK(hipStreamSynchronize(st_));
                st = (int)hpin[16];
            }
            if (st == kSpTimeout) return hand_off_timeout();
            if (st == kSpRunning) {                        // budget: a failed solve, like the host loop's
                const double rec_budget[2] = {(double)kSpBudget, (double)j};
                SPOK(hipMemcpyAsync(G.rec, rec_budget, sizeof(rec_budget), hipMemcpyHostToDevice, st_));
            }
            if (j > 0) guess = std::max(guess, std::min(j + 2, mx));
            if ((rc = evaluate())) return rc;
            launch_lm_decide(d_lm, d_scal, G.rec, d_chi_it, d_trials_it, DEFTRI_MAX_REPORT_ITERS, h_snap, -1, st_);
            SPOK(hipStreamSynchronize(st_));
            const LmState S2 = *h_snap;
            if (S2.last_its > 0) guess = std::max(2, S2.last_its + 2);
            if (S2.stop != 0) host_stop = true;
            continue;
        }
    }
    SPOK(hipStreamSynchronize(st_));
    for (hipEvent_t e : evpool) hipEventDestroy(e);
    LmState Lf;
    SPOK(hipMemcpy(&Lf, d_lm, sizeof(LmState), hipMemcpyDeviceToHost));
    const int nrep = std::min(Lf.it, (int)DEFTRI_MAX_REPORT_ITERS);
    if (nrep > 0) {
        SPOK(hipMemcpy(R.chi2_iter, d_chi_it, sizeof(double) * (size_t)nrep, hipMemcpyDeviceToHost));
        SPOK(hipMemcpy(R.trials_iter, d_trials_it, sizeof(int32_t) * (size_t)nrep, hipMemcpyDeviceToHost));
    }
    if (Lf.restore) {                                      // the last trial rejected: pop
        SPOK(hipMemcpyAsync(P.points, P.points_bak, sizeof(double) * 3 * (size_t)P.P, hipMemcpyDeviceToDevice, st_));
        SPOK(hipMemcpyAsync(P.scales, P.scales_bak, sizeof(double) * (size_t)P.S, hipMemcpyDeviceToDevice, st_));
        SPOK(hipMemcpyAsync(P.tg, P.tg_bak, sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToDevice, st_));
    }
    last_its = Lf.last_its > 0 ? Lf.last_its : last_its;
    R.trials_total += Lf.trials_total;
    R.trials_executed += Lf.trials_total;
    R.trials_rejected += Lf.trials_rejected;
    R.pcg_trials += Lf.pcg_trials;
    R.pcg_fallbacks += Lf.pcg_fail;
    R.pcg_iterations += Lf.pcg_iterations;
    R.status = Lf.stop == 2 ? DEFTRI_STATUS_TERMINATE : DEFTRI_STATUS_OK;
    R.iterations = Lf.it;
    R.lambda_final = Lf.lam;
    P.gate_lin = P.gate_trial = nullptr;
    G.gate = G.lgate = nullptr;
    G.lam_dev = nullptr;
    eval_chi2(analytic, 0, nullptr);
    SPOK(hipMemcpyAsync(hpin, d_scal, sizeof(double), hipMemcpyDeviceToHost, st_));
    SPOK(hipStreamSynchronize(st_));
    R.chi2_final = hpin[0];
    R.ms_linearize = -1.0;
    R.ms_pcg = -1.0;
    R.ms_factor = R.ms_solve = R.ms_update = -1.0;
    R.plan = DEFTRI_PLAN_ITERATIVE;
    R.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    return 0;
}

int SpSolver::solve_lm(const deftri_lm_params &prm, deftri_report &R) {
    if (!have_) return fail(DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(dev_);
    R.n_unknowns = G.ndof;
    R.rank = rank_;
    R.nranks = nranks_;
    R.lanes = 1;
    struct InLm {
        bool &f;
        explicit InLm(bool &x) : f(x) { f = true; }
        ~InLm() { f = false; }
    } in_lm(in_lm_);
    // the device-driven LM is opt-in (DEFTRI_DEVICE_LM=1): measured ~5 % slower than this loop at C2
    // (profiles/r04ab_lm_control.json) — a step that outruns its slot's guessed CG count costs the
    // slot in flight behind it, more than the host round trip per trial it saves
    static const bool dev_lm = std::getenv("DEFTRI_DEVICE_LM") != nullptr && std::getenv("DEFTRI_HOST_LM") == nullptr;
    if (!shard_ && dev_lm && !prm.verbose) return solve_lm_dev(prm, R);
    const bool dist = shard_;
    R.n_unknowns = G.ndof;
    R.rank = rank_;
    R.nranks = nranks_;
    R.lanes = 1;
    const int max_trials = prm.max_trials > 0 ? prm.max_trials : 10;
    const double tau = prm.tau > 0 ? prm.tau : 1e-5;
    const bool analytic = prm.analytic_jacobians != 0;
    auto t_start = std::chrono::steady_clock::now();
    int rc;
    if (!shard_ && (rc = save_entry())) return rc;     // (the sharded chain has no hand-off)
    eval_chi2(analytic, 0, nullptr);
    if (dist && (rc = tr_->allreduce(d_scal, 1, 0, st_))) return rc;
    SPOK(hipMemcpyAsync(hpin, d_scal, sizeof(double), hipMemcpyDeviceToHost, st_));
    SPOK(hipStreamSynchronize(st_));
    R.chi2_initial = hpin[0];
    double currentChi = R.chi2_initial;
    double lambda = 0, ni = 2;
    int status = DEFTRI_STATUS_OK, it;
    const int mx = budget();
    const int64_t nrec = kSpRecDoubles + (int64_t)kSpRed * (mx + 2);
    // the rank's share of dx.(lambda dx + b): its rows, plus the heavy dofs on rank 0 (contiguous
    // with rank 0's rows)
    const int64_t den_off = rank_ == 0 ? 0 : G.hd + 3 * (int64_t)G.row0;
    const int64_t den_n = rank_ == 0 ? G.hd + 3 * (int64_t)G.nown : 3 * (int64_t)G.nown;
    double t_lin = 0;
    // (one rank) the trial's sums are finished on the host; sharded, by the evaluation's last workgroup
    // before the all-reduce
    bool sums_pending = false;
    // DEFTRI_HOST_TIMING=1: the host's time from a trial's wait to the next launch call (a further
    // trial's setup or the next linearization) and the linearization's launch calls, per solve
    struct HostTiming {
        bool on = std::getenv("DEFTRI_HOST_TIMING") != nullptr, mark = false;
        std::chrono::steady_clock::time_point t_wait;
        double to_trial = 0, to_lin = 0, lin_issue = 0, trial_issue = 0;
        int n_trial = 0, n_lin = 0, n_issue = 0;
        double since() const { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_wait).count(); }
        ~HostTiming() {
            if (on)
                std::fprintf(stderr, "[deftri host] wait -> further trial %.1f us (%d), wait -> linearization %.1f us (%d), "
                             "linearization launch calls %.1f us per iteration, a trial's launch calls %.1f us\n",
                             n_trial ? to_trial / n_trial : 0.0, n_trial, n_lin ? to_lin / n_lin : 0.0, n_lin,
                             n_lin ? lin_issue / (n_lin + 1) : 0.0, n_issue ? trial_issue / n_issue : 0.0);
        }
    } ht;
    // one rank: k_trial_begin folded away — the backup into the trial's state update, the records'
    // clear into the evaluation (sharded: the prologue launch)
    const bool fold = !dist;
    if (fold) {                                   // the first trial's records start clear
        SPOK(hipMemsetAsync(G.rec, 0, sizeof(double) * (size_t)nrec, st_));
        SPOK(hipMemsetAsync(d_flag, 0, sizeof(int), st_));
    }
    for (it = 0; it < prm.n_iterations; it++) {
        auto t0 = std::chrono::steady_clock::now();
        bool ok;
        if (ht.on && ht.mark) { ht.to_lin += ht.since(); ht.n_lin++; ht.mark = false; }
        const auto tl0 = std::chrono::steady_clock::now();
        if ((rc = lin_iteration(analytic, it == 0, ok, !dist))) return rc;
        if (ht.on) ht.lin_issue += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tl0).count();
        double *chis = hpin;
        // (the host-added chi2 needs nothing from d_scal after iteration 0's max diag)
        if (it == 0 || !lin_host_pending_) SPOK(hipMemcpyAsync(chis, d_scal, sizeof(double) * 3, hipMemcpyDeviceToHost, st_));
        bool chi_pending = true;
        // (after a synchronization) the linearization's chi2: the host-added partials or d_scal[0]
        auto lin_chi = [&]() { return lin_host_pending_ ? lin_chi_host() : chis[0]; };
        if (it == 0) {
            SPOK(stream_wait(st_));
            currentChi = lin_chi();
            chi_pending = false;
            lambda = prm.user_lambda > 0 ? prm.user_lambda : tau * chis[2];
            ni = 2;
        }
        t_lin += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        double rho = 0;
        int qmax = 0;
        bool restore_pending = false;
        do {
            G.max_it = mx;
            G.tol2 = tol * tol;
            if (!fold) launch_trial_begin(P, d_flag, G.rec, nrec, st_, restore_pending);
            bool base_in_bak = restore_pending;   // (fold: the state update reads the backup)
            restore_pending = false;
            double *sc = hpin + 4;
            // update (x, halo rows from their owners), chi2 of the owned edges, the rank's share of
            // the rho denominator; one all-reduce of the two (sharded); one read-back
            auto evaluate = [&]() -> int {
                int r2;
                if (dist && (r2 = halo(3, G.x, false))) return r2;
                if (fold) {
                    launch_update_state_bak(P, G.x, base_in_bak, st_);
                    base_in_bak = true;                // a second evaluation starts from the backup
                } else {
                    launch_update_state(P, G.x, st_, nullptr);
                }
                SumJob den;
                den.n = den_n; den.a = G.x + den_off; den.b = G.b + den_off; den.lambda = lambda; den.mode = 1;
                den.out = d_scal + 1;
                if (!dist) {         // workgroup partials to the host, which finishes the sums
                    ReadBack rb;
                    rb.flag = d_flag; rb.rec = G.rec; rb.nrec = kSpRecDoubles; rb.h_flag = ipin; rb.h_rec = hpin + 16;
                    eval_chi2(analytic, 0, &den, &rb, h_epart_, G.rec, nrec);
                    sums_pending = true;
                    return 0;
                }
                eval_chi2(analytic, 0, &den);
                if ((r2 = tr_->allreduce(d_scal, 2, 0, st_))) return r2;
                launch_trial_readback(d_scal, 2, d_flag, G.rec, kSpRecDoubles, sc, ipin, hpin + 16, st_);
                return 0;
            };
            // after the stream synchronization that follows an evaluation: its sums, if the host finishes them
            auto finish_sums = [&]() {
                if (!sums_pending) return;
                double s4[4];
                trial_eval_host_sums(h_epart_, eval_nb_, s4);
                sc[0] = (s4[0] + s4[2]) + s4[1];
                sc[1] = s4[3];
                sums_pending = false;
            };
            auto t0p = std::chrono::steady_clock::now();
            if (ht.on && ht.mark) { ht.to_trial += ht.since(); ht.n_trial++; ht.mark = false; }
            const auto tt0 = std::chrono::steady_clock::now();
            if ((rc = cg_setup(lambda, G.b))) return rc;
            // CG iterations queued before the trial's evaluation: the last converged count + a
            // margin.  A short guess costs the evaluation, a state restore and a host round trip;
            // each extra queued iteration past convergence two early-out launches
            const int n = std::min(std::max(2, last_its + kSpGuessMargin), mx);
            if ((rc = cg_chain(lambda, 0, n))) return rc;
            int j = n;
            if ((rc = cg_tail(j, lambda))) return rc;
            if ((rc = evaluate())) return rc;
            if (ht.on) { ht.trial_issue += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tt0).count(); ht.n_issue++; }
            SPOK(stream_wait(st_));                 // the one host round trip of a trial (prediction held)
            if (ht.on) { ht.t_wait = std::chrono::steady_clock::now(); ht.mark = true; }
            finish_sums();
            if (chi_pending) { currentChi = lin_chi(); chi_pending = false; }
            int st = (int)hpin[16];
            if (st == kSpTimeout) return hand_off_timeout();
            bool solved = st == kSpConverged, evaluated = solved;
            int its = solved ? (int)hpin[17] : j;
            if (!solved) {
                R.pcg_continuations++;
                // restore the state the evaluation changed; continue the solve in chunks of 4
                SPOK(hipMemcpyAsync(P.points, P.points_bak, sizeof(double) * 3 * (size_t)P.P, hipMemcpyDeviceToDevice, st_));
                SPOK(hipMemcpyAsync(P.scales, P.scales_bak, sizeof(double) * (size_t)P.S, hipMemcpyDeviceToDevice, st_));
                SPOK(hipMemcpyAsync(P.tg, P.tg_bak, sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToDevice, st_));
                while (st == kSpRunning && j < mx) {
                    const int n2 = std::min(j + 4, mx);
                    if ((rc = cg_chain(lambda, j, n2))) return rc;
                    j = n2;
                    if ((rc = cg_tail(j, lambda))) return rc;
                    SPOK(hipMemcpyAsync(hpin + 16, G.rec, sizeof(double) * kSpRecDoubles, hipMemcpyDeviceToHost, st_));
                    SPOK(hipStreamSynchronize(st_));
                    st = (int)hpin[16];
                }
                if (st == kSpTimeout) return hand_off_timeout();
                solved = st == kSpConverged;
                its = solved ? (int)hpin[17] : j;
                if (fold && !solved) {                 // no evaluation clears this solve's records
                    SPOK(hipMemsetAsync(G.rec, 0, sizeof(double) * (size_t)nrec, st_));
                    SPOK(hipMemsetAsync(d_flag, 0, sizeof(int), st_));
                }
                if (solved) {
                    if ((rc = evaluate())) return rc;
                    SPOK(stream_wait(st_));
                    finish_sums();
                    evaluated = true;
                }
            }
            R.ms_pcg += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0p).count();
            R.pcg_iterations += its;
            step_its = its;
            step_solved = solved ? 1 : 0;
            if (solved) { R.pcg_trials++; last_its = its; }
            else R.pcg_fallbacks++;
            if (prm.verbose)
                std::fprintf(stderr, "[deftri/sp] rank %d pcg lambda %.6e iterations %d %s\n", rank_, lambda, its,
                             solved ? "converged" : "failed (trial rejected)");
            const double tempChi = (solved && evaluated) ? sc[0] : std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            const double scale = (solved && evaluated ? sc[1] : 0.0) + 1e-3;
            rho /= scale;
            R.trials_total++;
            R.trials_executed++;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                const double scaleFactor = std::max(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                restore_pending = true;                  // the next prologue (or the loop's end) restores
                R.trials_rejected++;
                if (!std::isfinite(lambda)) { qmax++; break; }
            }
            qmax++;
        } while (rho < 0 && qmax < max_trials);
        if (restore_pending) {
            SPOK(hipMemcpyAsync(P.points, P.points_bak, sizeof(double) * 3 * (size_t)P.P, hipMemcpyDeviceToDevice, st_));
            SPOK(hipMemcpyAsync(P.scales, P.scales_bak, sizeof(double) * (size_t)P.S, hipMemcpyDeviceToDevice, st_));
            SPOK(hipMemcpyAsync(P.tg, P.tg_bak, sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToDevice, st_));
        }
        if (it < DEFTRI_MAX_REPORT_ITERS) { R.chi2_iter[it] = currentChi; R.trials_iter[it] = qmax; }
        if (prm.verbose)
            std::fprintf(stderr, "[deftri/sp] it %d chi2 %.9e lambda %.6e trials %d\n", it, currentChi, lambda, qmax);
        if (qmax == max_trials || rho == 0 || !std::isfinite(lambda)) { status = DEFTRI_STATUS_TERMINATE; it++; break; }
    }
    eval_chi2(analytic, 0, nullptr);
    if (dist && (rc = tr_->allreduce(d_scal, 1, 0, st_))) return rc;
    SPOK(hipMemcpyAsync(hpin, d_scal, sizeof(double), hipMemcpyDeviceToHost, st_));
    SPOK(hipStreamSynchronize(st_));
    R.chi2_final = hpin[0];
    R.status = status;
    R.iterations = it;
    R.lambda_final = lambda;
    R.ms_linearize = t_lin;
    R.ms_factor = R.ms_solve = R.ms_update = -1.0;           // no factorization; not split
    R.plan = DEFTRI_PLAN_ITERATIVE;
    R.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    return 0;
}

int SpSolver::download(double *points, double *scales, double *tg) {
    if (!have_) return fail(DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(dev_);
    SPOK(hipStreamSynchronize(st_));
    if (points) {
        std::vector<double> h(3 * (size_t)P.P);
        SPOK(hipMemcpy(h.data(), P.points, sizeof(double) * h.size(), hipMemcpyDeviceToHost));
        for (int32_t p = 0; p < P.P; p++)
            for (int c = 0; c < 3; c++) points[3 * (size_t)p + c] = h[3 * (size_t)H.row_of_point[p] + c];
    }
    if (scales) SPOK(hipMemcpy(scales, P.scales, sizeof(double) * (size_t)P.S, hipMemcpyDeviceToHost));
    if (tg) SPOK(hipMemcpy(tg, P.tg, sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToHost));
    return 0;
}

int SpSolver::reset_state() {
    if (!have_) return fail(DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(dev_);
    SPOK(hipMemcpyAsync(P.points, init_[0], sizeof(double) * 3 * (size_t)P.P, hipMemcpyDeviceToDevice, st_));
    SPOK(hipMemcpyAsync(P.scales, init_[1], sizeof(double) * (size_t)P.S, hipMemcpyDeviceToDevice, st_));
    SPOK(hipMemcpyAsync(P.tg, init_[2], sizeof(double) * 7 * (size_t)P.Q, hipMemcpyDeviceToDevice, st_));
    SPOK(hipStreamSynchronize(st_));
    return 0;
}

int SpSolver::chi2(double *out) {
    if (!have_) return fail(DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(dev_);
    eval_chi2(true, 0, nullptr);
    int rc;
    if (shard_ && (rc = tr_->allreduce(d_scal, 1, 0, st_))) return rc;
    SPOK(hipMemcpyAsync(hpin, d_scal, sizeof(double), hipMemcpyDeviceToHost, st_));
    SPOK(hipStreamSynchronize(st_));
    *out = hpin[0];
    return 0;
}

int SpSolver::gradient(double *b, double *hdiag, int64_t n, bool analytic) {
    if (!have_) return fail(DEFTRI_E_NOPROBLEM, "no problem uploaded");
    if (nranks_ > 1) return fail(DEFTRI_E_ARG, "not available on a point-sharded context");
    if (n != G.ndof) return fail(DEFTRI_E_ARG, "size mismatch");
    hipSetDevice(dev_);
    bool ok;
    int rc = lin_iteration(analytic, false, ok);
    if (rc) return rc;
    if (b) {
        sp_launch_permute_out(G.P, G.hd, d_row_of_point, G.b, d_tmp, st_);
        SPOK(hipMemcpyAsync(b, d_tmp, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, st_));
    }
    SPOK(hipStreamSynchronize(st_));
    if (hdiag) {
        std::vector<double> hv(6 * (size_t)G.nown), hl(21 * (size_t)G.Q + G.S);
        SPOK(hipMemcpy(hv.data(), G.Hv, sizeof(double) * hv.size(), hipMemcpyDeviceToHost));
        SPOK(hipMemcpy(hl.data(), G.hl, sizeof(double) * hl.size(), hipMemcpyDeviceToHost));
        const int diag3[3] = {0, 2, 5};
        for (int32_t q = 0; q < G.Q; q++)
            for (int a = 0; a < 6; a++) hdiag[6 * q + a] = hl[21 * (size_t)q + a * (a + 1) / 2 + a];
        for (int32_t s = 0; s < G.S; s++) hdiag[6 * G.Q + s] = hl[21 * (size_t)G.Q + s];
        for (int32_t p = 0; p < G.P; p++) {
            const int32_t l = H.row_of_point[p] - H.lo;
            for (int c = 0; c < 3; c++) hdiag[G.hd + 3 * (int64_t)p + c] = hv[6 * (size_t)l + diag3[c]];
        }
    }
    return 0;
}

int SpSolver::damped_solve(double lambda, const double *rhs, double *x, int64_t n) {
    if (!have_) return fail(DEFTRI_E_NOPROBLEM, "no problem uploaded");
    if (nranks_ > 1) return fail(DEFTRI_E_ARG, "not available on a point-sharded context");
    if (n != G.ndof) return fail(DEFTRI_E_ARG, "size mismatch");
    hipSetDevice(dev_);
    bool ok;
    int rc = lin_iteration(true, false, ok);
    if (rc) return rc;
    SPOK(hipMemcpyAsync(d_dx0, rhs, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, st_));
    sp_launch_permute_in(G.P, G.hd, d_row_of_point, d_dx0, d_tmp, st_);
    bool solved = false;
    int its = 0;
    if ((rc = pcg_solve(lambda, d_tmp, solved, its))) return rc;
    sp_launch_permute_out(G.P, G.hd, d_row_of_point, G.x, d_dx0, st_);
    SPOK(hipMemcpyAsync(x, d_dx0, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, st_));
    SPOK(hipStreamSynchronize(st_));
    if (!solved) return fail(DEFTRI_E_NUMERIC, "PCG did not converge within its budget (" + std::to_string(its) + " iterations)");
    return 0;
}

// y = (H + lambda I) x with the CG chain's own product kernels (the three-launch form: phase 1,
// phase 2, the heavy finish), H linearized at the current state with the analytic Jacobians as
// gradient() / damped_solve() do: the operator the solves invert, for their backward errors
int SpSolver::hessian_product(double lambda, const double *x, double *y, int64_t n) {
    if (!have_) return fail(DEFTRI_E_NOPROBLEM, "no problem uploaded");
    if (nranks_ > 1) return fail(DEFTRI_E_ARG, "not available on a point-sharded context");
    if (n != G.ndof) return fail(DEFTRI_E_ARG, "size mismatch");
    hipSetDevice(dev_);
    bool ok;
    int rc = lin_iteration(true, false, ok);
    if (rc) return rc;
    SPOK(hipMemcpyAsync(d_dx0, x, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, st_));
    sp_launch_permute_in(G.P, G.hd, d_row_of_point, d_dx0, d_tmp, st_);
    sp_launch_load_p(G.ndof, d_tmp, G.zp, st_);
    // iteration 0 runs (r.r = 1 > 0), beta = 0 so p = z = x; every partial to plain stores
    SPOK(hipMemsetAsync(G.rec, 0, sizeof(double) * (size_t)(kSpRecDoubles + 2 * kSpRed), st_));
    const double one = 1.0;
    SPOK(hipMemcpyAsync(G.red + 1, &one, sizeof(double), hipMemcpyHostToDevice, st_));
    SpDev g = G;
    g.merged = 0; g.fuse = 0; g.fuse_heavy = 0; g.tparts = 0;
    g.max_it = 1;
    g.tol2 = 0.0;
    if (G.tile) {                                  // the fused product + its cross slots and heavy sums
        sp_launch_tile_product(g, lambda, fp32_jac != 0, st_);
    } else {
        sp_launch_product(g, 0, lambda, fp32_jac != 0, st_);
        sp_launch_heavy(g, 0, lambda, 0, st_);
    }
    sp_launch_permute_out(G.P, G.hd, d_row_of_point, G.q, d_dx0, st_);
    SPOK(hipMemcpyAsync(y, d_dx0, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, st_));
    SPOK(hipStreamSynchronize(st_));
    SPOK(hipMemsetAsync(G.rec, 0, sizeof(double) * (size_t)(kSpRecDoubles + 2 * kSpRed), st_));
    return 0;
}

// one trial's kernels under the caller's profiler: linearize + lin, then (after an unprofiled solve
// that learns the iteration count) the setup and exactly that many CG iterations
int SpSolver::profile_trial(double lambda, KProf &prof, bool analytic) {
    if (!have_) return fail(DEFTRI_E_NOPROBLEM, "no problem uploaded");
    hipSetDevice(dev_);
    SPOK(hipStreamSynchronize(st_));
    set_profiler(&prof);
    bool ok;
    int rc = lin_iteration(analytic, false, ok, !shard_);   // (the host loop's launches)
    set_profiler(nullptr);
    if (rc) return rc;
    bool solved = false;
    int its = 0;
    if ((rc = pcg_solve(lambda, G.b, solved, its))) return rc;
    set_profiler(&prof);
    SPOK(hipMemsetAsync(G.rec, 0, sizeof(double) * (size_t)(kSpRecDoubles + kSpRed * (G.max_it + 2)), st_));
    rc = cg_setup(lambda, G.b);
    if (!rc) rc = cg_chain(lambda, 0, its);
    if (!rc) rc = cg_tail(its, lambda);
    if (!rc && !shard_) {               // the trial's evaluation (of the current state: no update)
        SumJob den;
        den.n = G.hd + 3 * (int64_t)G.nown; den.a = G.x; den.b = G.b; den.lambda = lambda; den.mode = 1;
        den.out = d_scal + 1;
        rc = eval_chi2(analytic, 0, &den, nullptr, h_epart_);
    }
    set_profiler(nullptr);
    if (rc) return rc;
    SPOK(hipStreamSynchronize(st_));
    step_its = its;
    step_solved = solved ? 1 : 0;
    return 0;
}

int SpSolver::vertex_owner(int32_t *owner, int64_t nv) const {
    if (nv != (int64_t)G.Q + G.S + G.P) return DEFTRI_E_ARG;
    for (int32_t k = 0; k < G.Q + G.S; k++) owner[k] = 0;
    for (int32_t p = 0; p < G.P; p++) {
        const int32_t r = H.row_of_point[p];
        int o = (int)(std::upper_bound(H.rank_row_begin.begin(), H.rank_row_begin.end(), r) - H.rank_row_begin.begin()) - 1;
        owner[G.Q + G.S + p] = std::max(0, std::min(o, nranks_ - 1));
    }
    return 0;
}

}  // namespace deftri
