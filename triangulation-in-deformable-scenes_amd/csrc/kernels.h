// kernels.h — device-side problem / plan views and kernel launchers (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace deftri {

constexpr int64_t kHeavyChunks = 16;   // chunk count above which an H block / b vertex is reduced by a workgroup

// problem arrays resident in HBM (layout = deftri_problem_desc, SoA)
struct DevProblem {
    int32_t P = 0, Q = 0, S = 0, C = 0, R = 0, D = 0, E = 0, NR = 0;
    // state
    double *points = nullptr, *scales = nullptr, *tg = nullptr;
    double *points_bak = nullptr, *scales_bak = nullptr, *tg_bak = nullptr;
    // cameras
    float *cam_kb8 = nullptr;
    double *cam_pose = nullptr, *cam_R = nullptr;
    // edges
    int32_t *rep_point = nullptr, *rep_cam = nullptr;
    double *rep_obs = nullptr, *rep_info = nullptr;
    double huber_delta = 0;
    int32_t *dep_point = nullptr, *dep_scale = nullptr, *dep_cam = nullptr;
    double *dep_meas = nullptr, *dep_info = nullptr;
    int32_t *arap_pts = nullptr, *arap_pair = nullptr, *arap_rot = nullptr;
    double *arap_w = nullptr, *rot = nullptr, *pair_area = nullptr, *pair_info = nullptr;
    // linearization
    double *Jrep = nullptr, *Wrep = nullptr, *Erep = nullptr, *chi_rep = nullptr;
    double *Jdep = nullptr, *Wdep = nullptr, *Edep = nullptr, *chi_dep = nullptr;
    double *Jarap = nullptr, *Warap = nullptr, *Earap = nullptr, *chi_arap = nullptr;
    int64_t jarap_ld = 0;       // 0: J per edge contiguous ([E][18], the multifrontal plan's kernels);
                                // > 0: column-major [18][jarap_ld] (the iterative plan: coalesced loads)
    double *tg_pre = nullptr;   // per pair: T_g and its 12 numeric-Jacobian perturbations (k_arap_pre)
    // device-driven LM (spcg_solver.cpp, one rank): kernels return at once when their gate word is 0 —
    // gate_lin for the linearization's launches, gate_trial for a trial's; nullptr: always run
    const int *gate_lin = nullptr, *gate_trial = nullptr;
    // the linearization's chi2 as per-workgroup partials (the iterative plan, one rank): set, k_lin_pts'
    // reprojection / depth workgroups and k_lin_arap's workgroups over the first n_arap_sum edges store
    // their sums at lin_part[b] (lin_chi_blocks' layout) instead of per-edge chi2 — pinned host memory
    // (the host adds them after its synchronization) or HBM (launch_part_sums adds them)
    double *lin_part = nullptr;
    int64_t n_arap_sum = 0;
};

struct FrontDev {
    const int32_t *m, *s, *parent, *nchild, *child0, *child1, *direct, *rhs_bnd, *panel_off;
    const int64_t *arena_off, *vec_off, *rows_off, *bmap_off, *inv_off;
    const int32_t *rows, *bmap;
};

struct LevelDev {
    int64_t ea_off[2]; int32_t nea[2];
    struct Step { int64_t diag_off; int32_t ndiag; int64_t trsm_off; int32_t ntrsm; int64_t upd_off; int32_t nupd; int32_t k0, kA, kmax, inner, stream, wait_side; double upd_flops; int32_t ntail, ndiag_tail; };
    std::vector<Step> steps;
    int64_t fwd_off; int32_t nfwd;
    struct SolveStep { int64_t off; int32_t n; };
    std::vector<SolveStep> fsteps, bsteps;
    int64_t bgemv_off; int32_t nbgemv;
    int64_t fchain_off; int32_t nfchain;
    int64_t bchain_off; int32_t nbchain;
};

// batched LM trials ("lambda lanes"): every factor/solve launch carries a second grid dimension,
// lane = blockIdx.y, whose buffers sit at these strides from lane 0's (all zero for one lane)
constexpr int kMaxLanes = 8;
// status flag bits: 1 = zero pivot (the trial fails, as g2o's); kStatusWaitTimeout = a fused-TRSM tile
// gave up waiting for its panel (a plan / dispatch bug: the solve reports DEFTRI_E_HIP).  Large so a
// cross-rank sum of zero-pivot flags never reaches it.
constexpr int kStatusWaitTimeout = 1 << 20;
struct LaneOff {
    int64_t arena = 0, inv = 0, vec = 0, x = 0;   // doubles between consecutive lanes' buffers
    int64_t pflag = 0;                            // panels between consecutive lanes' flags (x 4096: wbuf doubles)
    double lam[kMaxLanes] = {0, 0, 0, 0, 0, 0, 0, 0};   // setLambda of each lane (k_scatter)
};

struct DevPlan {
    int64_t nv = 0, ndof = 0;
    int64_t *voff = nullptr;
    int32_t *vdim = nullptr;
    // H blocks
    int64_t nblocks = 0, hval_size = 0;
    double *hval = nullptr;
    int64_t *blk_val_off = nullptr, *blk_arena = nullptr;
    int32_t *blk_rows = nullptr, *blk_cols = nullptr, *blk_ld = nullptr, *blk_diag = nullptr;
    int64_t *blk_row_dof = nullptr, *blk_col_dof = nullptr;     // diagnostics (H x)
    int64_t nhchunks = 0;
    uint64_t *hcontrib = nullptr;
    int64_t *hchunk_begin = nullptr, *hblk_chunk_begin = nullptr;
    int32_t *hchunk_len = nullptr;
    double *hpart = nullptr;
    int64_t nheavy_h = 0, nheavy_b = 0;
    int64_t *heavy_h = nullptr, *heavy_b = nullptr;     // blocks / vertices with > kHeavyChunks chunks
    double *heavy_scratch = nullptr;                     // per heavy item x 32 slices x 36 partial sums
    int64_t nbchunks = 0;
    uint64_t *bcontrib = nullptr;
    int64_t *bchunk_begin = nullptr, *bv_chunk_begin = nullptr;
    int32_t *bchunk_len = nullptr;
    double *bpart = nullptr;
    double *b = nullptr;
    // factor
    int64_t arena_size = 0, vec_size = 0;
    int64_t inv_size = 0;
    double *inv = nullptr;       // panel-triangle inverses (Front::inv_off)
    double *arena = nullptr, *vec = nullptr, *yvec = nullptr;   // yvec: forward solution y per front row
    FrontDev fd{};
    int32_t *tasks = nullptr;
    std::vector<LevelDev> levels;
    int *flag = nullptr;          // one status flag per lane (1 zero pivot, kStatusWaitTimeout)
    int64_t npanels = 0;
    int *pflag = nullptr;         // per panel (x lanes): the factorization epoch that last factored it
    double *wbuf = nullptr;       // per panel (x lanes): 64 x 64 TRSM operand W = Linv^T D^{-1} (fused TRSM)
    int nlanes = 1;               // lanes the factor / solve launches cover (blockIdx.y)
    int f32_update = 0;           // 1: trailing updates on fp32 MFMA (deftri_set_factor_precision)
    LaneOff lo{};
};

// per-launch device timing for deftri_profile_trial (never active on the solve path)
struct KProfRec { const char *name; hipEvent_t e0, e1; unsigned grid; double work; int level; };
struct KProf {
    std::vector<hipEvent_t> pool;
    size_t next = 0;
    std::vector<KProfRec> recs;
};
void set_profiler(KProf *p);
bool profiling();
hipEvent_t prof_begin(hipStream_t st);   // nullptr unless profiling
void prof_end(const char *name, hipEvent_t e0, unsigned grid, double work, hipStream_t st);

void launch_linearize(const DevProblem &P, hipStream_t st, bool want_jac, bool analytic);
void launch_assemble(const DevProblem &P, const DevPlan &L, hipStream_t st);
// lam_dev (optional): lambda read on the device (captured graphs); otherwise the argument / L.lo.lam
void launch_scatter(const DevPlan &L, double lambda, hipStream_t st, const double *lam_dev = nullptr);   // one lane
void launch_scatter_lanes(const DevPlan &L, hipStream_t st, const double *lam_dev = nullptr);         // L.nlanes lanes
// point-sharded plan: called by launch_factor before level h (contribution blocks from other ranks),
// by launch_solve before forward level h and after backward level h (DistPlan transfers of that level)
enum { kHookFactor = 0, kHookForward = 1, kHookBackward = 2 };
typedef void (*LevelHook)(void *user, int phase, int level);
void launch_factor(const DevPlan &L, hipStream_t st, hipStream_t side, hipEvent_t *ev, int nev,
                   LevelHook hook = nullptr, void *hook_user = nullptr);
void launch_solve(const DevPlan &L, const double *rhs, double *x, hipStream_t st, const double *bpart = nullptr,
                  LevelHook hook = nullptr, void *hook_user = nullptr);
void launch_update_state(const DevProblem &P, const double *dx, hipStream_t st, const int *flag = nullptr);
// a trial's prologue: state backup (restore: the state restored from the backup), zero-pivot flag and
// nzero doubles at `zero` cleared, one launch
// The device-driven LM (one rank, iterative plan; spcg_solver.cpp SpSolver::solve_lm_dev): the
// variables of g2o's OptimizationAlgorithmLevenberg::solve (reference g2oBundleAdjustment.cc:959-962,
// SURVEY Appendix A) in HBM, so the host queues trial slots without reading each trial's outcome.
// A slot = [linearization (gate_lin)] [prologue] [setup + CG + evaluation (gate_trial)] [decide].
struct LmState {
    double lam, ni, cur, rho;            // _currentLambda, _ni, currentChi, the last trial's rho
    int32_t gate_trial, gate_lin;        // the next slot's gates (read by every gated kernel)
    int32_t it, q;                       // LM iteration, trials of it so far (g2o's qmax)
    int32_t stop;                        // 0 running, 1 n_iterations done, 2 g2o Terminate, 3 PCG step unfinished,
                                         // 4 alpha hand-off timeout (an error, raised by the host)
    int32_t restore;                     // the last trial was rejected: the next prologue restores the state
    int32_t need_lin;                    // the next slot starts a new iteration
    int32_t slot;                        // the enqueue index of the last slot decided
    int32_t trials_total, trials_rejected, pcg_trials, pcg_fail;
    int32_t last_its, n_it, max_trials, stop_slot;   // stop_slot: the enqueue index that set stop
    int64_t pcg_iterations;
};
// the device-driven LM's prologue: gate_trial 0 -> nothing; else the backup (or, restore != 0,
// the restore) and the cleared records, as launch_trial_begin; thread 0 also folds the linearization
// just run (gate_lin) into the LM state: current chi2 = scal[0], and at iteration 0 lambda = tau max diag
void launch_trial_begin_dev(const DevProblem &P, int *flag, double *zero, int64_t nzero, LmState *lm, const double *scal,
                            double tau, double user_lambda, hipStream_t st);
// the device-driven LM's decision after a slot's evaluation (one thread): rho, accept / reject, the
// lambda / nu update, g2o's loop and Terminate conditions, the per-iteration report, the next slot's
// gates; a PCG step still running stops the slots for the host (stop 3).  A copy of the state goes
// to pinned host memory (`snap`).  `slot`: the enqueue index (-1 for the host's continuation).
void launch_lm_decide(LmState *lm, const double *scal, const double *rec, double *chi_it, int32_t *trials_it, int max_report,
                      LmState *snap, int slot, hipStream_t st);
void launch_trial_begin(const DevProblem &P, int *flag, double *zero, int64_t nzero, hipStream_t st,
                        bool restore = false);
// a trial's read-back: ns scalars, the flag and (rec != nullptr) nrec record values into pinned host memory
void launch_trial_readback(const double *scal, int ns, const int *flag, const double *rec, int nrec, double *h_scal,
                           int *h_flag, double *h_rec, hipStream_t st);
void launch_sum(int64_t n, const double *a, const double *b, double lambda, int mode, double *part, int nparts,
                double *out, hipStream_t st, const double *w = nullptr);
// several fixed-order sums in two launches (the per-array arithmetic of launch_sum: the same
// partials and final butterfly), optionally total = (out0 + out2) + out1 — the order launch_sum's
// three-value pass adds them in
// lambda_dev (when set) replaces lambda: the damping the device-driven LM keeps in HBM
struct SumJob { int64_t n = 0; const double *a = nullptr, *b = nullptr, *w = nullptr; double lambda = 0; int mode = 0; double *out = nullptr;
                const double *lambda_dev = nullptr; };
constexpr int kMaxSumJobs = 4;
struct SumJobs { SumJob j[kMaxSumJobs]; int nj = 0; double *total = nullptr; const int *gate = nullptr; };
void launch_sum_multi(const SumJobs &J, double *part, int nparts, hipStream_t st);
// the trial read-back (k_trial_readback) folded into launch_sum_multi_fused's last workgroup
struct ReadBack {
    const double *scal = nullptr; int ns = 0; const int *flag = nullptr; const double *rec = nullptr; int nrec = 0;
    double *h_scal = nullptr; int *h_flag = nullptr; double *h_rec = nullptr;
};
// launch_sum_multi in one launch (same sums, same order; *cnt zero between launches), optionally
// followed by the read-back
void launch_sum_multi_fused(const SumJobs &J, double *part, int nparts, int *cnt, const ReadBack &rb, hipStream_t st);
// the errors and chi2 of all edges (launch_linearize without Jacobians) in one launch
void launch_lin_chi(const DevProblem &P, hipStream_t st);
// a trial's evaluation in one launch (launch_lin_chi + launch_sum_multi_fused without the per-edge
// chi2 arrays): each workgroup sums the chi2 of a run of reprojection / depth / owned ARAP edges,
// or a run of dx.(lambda dx + b), into its partial; the last workgroup (ticket) adds each kind's
// partials in order into out[0..2] (rep, dep, arap), den_out and total = (rep + arap) + dep, then
// the read-back.  The sums' order is this launch's own: every caller of the trial's evaluation
// uses it.  *cnt zero between launches.
struct EvalJob {
    int64_t n_arap = 0;                          // the edges whose chi2 is summed (the owned ones)
    const double *dx = nullptr, *b = nullptr;    // n_den > 0: den_out = sum dx (lambda dx + b)
    int64_t n_den = 0;
    double lambda = 0;
    const double *lambda_dev = nullptr;          // replaces lambda (the device-driven LM)
    double *out = nullptr, *den_out = nullptr, *total = nullptr;
    const int *gate = nullptr;
    // set: each workgroup stores its partial into this pinned host array and workgroup 0 does the
    // read-back's record / flag copies; no ticket, no device sums — the host finishes the sums after
    // its stream synchronization (trial_eval_host_sums, the last workgroup's order)
    double *h_part = nullptr;
    // with h_part: after its read-back copies, workgroup 0 clears the solve records (nclear doubles) and
    // the flag — k_trial_begin's clears, for the next trial — when the record's status word is final
    // (a running solve is continued by the host and keeps its records)
    double *rec_clear = nullptr;
    int64_t nclear = 0;
    int *flag_clear = nullptr;
};
// the trial's state update with k_trial_begin's backup folded in: base = the backup (restore: after a
// rejected trial, or a second evaluation of the same trial) or the current state; backup = base (not
// restore); state = base + dx (k_update_state's arithmetic)
void launch_update_state_bak(const DevProblem &P, const double *dx, bool restore, hipStream_t st);
// the workgroup counts of the four kinds (rep, dep, arap, den) of a trial evaluation
void trial_eval_blocks(const DevProblem &P, const EvalJob &J, int nb[4]);
// the four sums from the host partials, in the device's final order (per kind: lane l adds partials
// l, l + 64, ... in order, then the xor butterfly 32 .. 1; lane 0's value)
void trial_eval_host_sums(const double *h_part, const int nb[4], double out[4]);
// the linearization's chi2 partial layout (DevProblem::lin_part): rep, dep, arap workgroup counts
void lin_chi_blocks(const DevProblem &P, int nb[4]);
// one workgroup: the four sums of a partial layout in trial_eval_host_sums' order into out[0..2],
// den_out (nb[3] > 0), total = (out0 + out2) + out1; gated like the linearization (gate)
void launch_part_sums(const double *part, const int nb[4], double *out, double *den_out, double *total, const int *gate,
                      hipStream_t st);
// edges per thread of a trial evaluation's workgroup (DEFTRI_EVAL_EPT, 1..8; default 2)
int eval_edges_per_thread();
// the partial slots launch_trial_eval needs (part's length)
int64_t trial_eval_parts(const DevProblem &P, const EvalJob &J);
void launch_trial_eval(const DevProblem &P, const EvalJob &J, double *part, int *cnt, const ReadBack &rb, hipStream_t st);
void launch_pack_cb(const DevPlan &L, int64_t arena_off, int m, int s, double *buf, hipStream_t st);
void launch_ea_packed(const DevPlan &L, int64_t ea_off, int nea, const double *buf, hipStream_t st);
void launch_gather_idx(int n, const int32_t *idx, const double *src, double *dst, hipStream_t st);
void launch_scatter_idx(int n, const int32_t *idx, const double *src, double *dst, hipStream_t st);
void launch_diag_entries(const DevPlan &L, double *diagv, hipStream_t st);
void launch_absmax(int64_t n, const double *a, double *part, int nparts, double *out, hipStream_t st);
void launch_int_to_double(int n, const int *a, double *out, hipStream_t st);
void launch_maxdiag(const DevPlan &L, double *part, int nparts, double *out, hipStream_t st);
// calculatePixelsStandDev partial sums (metrics.hip): 8 doubles per 256-match block
void launch_pixel_partials(int nblk, const int32_t *blk_first, const int32_t *blk_last, const int32_t *blk_pair,
                           const int32_t *pair_cams, const float *cams, const float *pts, const float *obs,
                           double *part, hipStream_t st);
// Mapping::triangulateSimulatedMapPoints, NRSLAM / FarPoints (triangulate.hip)
void launch_triangulate_nrslam(int n, const float *uv1, const float *uv2, const float *kb1, const float *kb2,
                               const float *Tp, float min_cos, float *x1, float *x2, uint8_t *valid, hipStream_t st);
void launch_hmul(const DevPlan &L, const int64_t *brow_dof, const int64_t *bcol_dof, const double *x, double *y,
                 int64_t n, hipStream_t st);

}  // namespace deftri
