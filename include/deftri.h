/*
 * deftri.h — C-ABI of the MI355X-native deformable-triangulation LM solver.
 *
 * This is the drop-in boundary for the hot path of
 * luicalrob/Triangulation-in-Deformable-Scenes: the g2o Levenberg–Marquardt
 * solve inside `arapOptimization` (Modules/Optimization/g2oBundleAdjustment.cc:608-1008
 * at the surveyed revision; the LM call is `optimizer.optimize(nOptIterations)`
 * at g2oBundleAdjustment.cc:962), and the BlockSolver_6_3 Schur LM of its BA entry
 * points (:38-444).  The reference's C++ entry points (Modules/Optimization/g2oBundleAdjustment.h:36-75)
 * are mirrored by deftri/optimization.py and deftri/ba.py; the adapter a C++ maintainer would put
 * behind those signatures is shown in INTEGRATION.md.  Both sit on this plain C interface.
 *
 * Conventions
 *  - every function returns int: 0 = OK, < 0 = error (see DEFTRI_E_*); the message
 *    of the last error on a context is available from deftri_last_error().
 *  - host arrays are owned by the caller and only read (or written, for outputs)
 *    during the call; device buffers are owned by the context.
 *  - one context per host thread; contexts are independent.
 *  - no C++ exceptions cross this boundary.
 *
 * Problem layout ("graph descriptor"): the flattened g2o graph that
 * arapOptimization builds (g2oBundleAdjustment.cc:640-953) — see DESIGN.md §2.
 *   vertices : points (3 dof, VertexSBAPointXYZ, g2oTypes.h:39-56),
 *              per KF-pair one SE3 T_g (g2o::VertexSE3Expmap, 6 dof, T <- exp(d)*T)
 *              and per KF-pair two depth scales (VertexDepthScale, g2oTypes.h:78-94)
 *   edges    : reprojection  EdgeSE3ProjectXYZPerKeyFrameOnlyPoints (g2oTypes.h:267-298),
 *              depth         EdgeDepthCorrection (g2oTypes.h:390-421),
 *              ARAP          EdgeARAP (g2oTypes.h:300-349).
 */
#ifndef DEFTRI_H
#define DEFTRI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DEFTRI_ABI_VERSION 8

/* error codes */
#define DEFTRI_OK             0
#define DEFTRI_E_ARG         -1   /* invalid argument / inconsistent descriptor */
#define DEFTRI_E_HIP         -2   /* HIP runtime error (allocation, launch) */
#define DEFTRI_E_NOPROBLEM   -3   /* solve/download before upload */
#define DEFTRI_E_NUMERIC     -4   /* non-finite state */
#define DEFTRI_E_NODEVICE    -5   /* no usable gfx950 device */
#define DEFTRI_E_GRAPH       -6   /* graph construction failed (e.g. < 3 mesh points) */
#define DEFTRI_E_SEARCH      -7   /* the weight search ended on a failure code (nlopt::opt::optimize
                                     throws there, g2oBundleAdjustment.cc:515): the round is not run */

/* solver status written into deftri_report.status (g2o SparseOptimizer::optimize semantics) */
#define DEFTRI_STATUS_OK         0  /* ran all requested iterations */
#define DEFTRI_STATUS_TERMINATE  1  /* g2o "Terminate": 10 failed trials, rho == 0 or lambda not finite */

typedef struct deftri_ctx deftri_ctx;

/* Flattened non-rigid BA / ARAP problem (all indices are 0-based). */
typedef struct deftri_problem_desc {
    int32_t n_points;   /* P   point vertices, 3 dof each                                  */
    int32_t n_pairs;    /* Q   KF pairs: one SE3 T_g vertex each                            */
    int32_t n_scales;   /* S   depth-scale vertices (reference: 2 per pair)                 */
    int32_t n_cams;     /* C   fixed camera poses / calibrations used by the edges          */
    int32_t n_rep;      /* R   reprojection edges                                           */
    int32_t n_depth;    /* D   depth edges                                                  */
    int32_t n_arap;     /* E   ARAP edges (directed, as the reference inserts them)         */
    int32_t n_rot;      /* rows of the per-mesh-vertex rotation table R_i                   */

    /* initial state */
    const double *points;     /* [P*3]  VertexSBAPointXYZ estimates                         */
    const double *tg;         /* [Q*7]  SE3Quat per pair: qx qy qz qw tx ty tz              */
    const double *scales;     /* [S]    VertexDepthScale estimates                           */

    /* cameras (fixed): Kannala–Brandt8 params and pose T_cw (g2o::SE3Quat of the KF pose)   */
    const float  *cam_kb8;    /* [C*8]  fx fy cx cy k0 k1 k2 k3 (KannalaBrandt8.cc:22-29)   */
    const double *cam_pose;   /* [C*7]  qx qy qz qw tx ty tz                                */

    /* reprojection edges: e = obs - KB8(T_cw * p), info = invSigma2(octave)*repW * I2,
       Huber(delta) — g2oBundleAdjustment.cc:765-812                                          */
    const int32_t *rep_point; /* [R] */
    const int32_t *rep_cam;   /* [R] */
    const double  *rep_obs;   /* [R*2] */
    const double  *rep_info;  /* [R]  scalar multiple of I2 */
    double huber_delta;       /* robust kernel delta (reference: (float)sqrt(100.991)); <= 0 disables */

    /* depth edges: e = (d/s - (T_cw p)_z)^2 (x500 if s <= 0), info = 1/sigma^2
       — g2oTypes.h:403-417, g2oBundleAdjustment.cc:816-856                                   */
    const int32_t *dep_point; /* [D] */
    const int32_t *dep_scale; /* [D] */
    const int32_t *dep_cam;   /* [D] */
    const double  *dep_meas;  /* [D] */
    const double  *dep_info;  /* [D] */

    /* ARAP edges (g2oTypes.h:311-342): vertices (p1_i, p2_i, p1_j, p2_j, T_g[pair]),
       R_i = rot[arap_rot[2e]], R_j = rot[arap_rot[2e+1]], w_ij = arap_w[e],
       area = pair_area[pair], info = pair_info[pair] (= arapW * T^2, :946)                 */
    const int32_t *arap_pts;  /* [E*4] */
    const int32_t *arap_pair; /* [E]   */
    const int32_t *arap_rot;  /* [E*2] */
    const double  *arap_w;    /* [E]   */
    const double  *rot;       /* [n_rot*9] row-major 3x3 */
    const double  *pair_area; /* [Q] */
    const double  *pair_info; /* [Q] */

    /* optional: 2-D ordering coordinates per point (the mesh plane).  NULL = use points x,y.
       Only affects the fill-reducing ordering of the sparse LDL^T, never the result's meaning. */
    const double *order_xy;   /* [P*2] or NULL */
} deftri_problem_desc;

typedef struct deftri_lm_params {
    int32_t n_iterations;   /* g2o optimize(n) */
    int32_t max_trials;     /* g2o _maxTrialsAfterFailure (default 10) */
    double  tau;            /* lambda init = tau * max diag(H) (default 1e-5) */
    double  user_lambda;    /* > 0: use as initial lambda (g2o _userLambdaInit) */
    int32_t analytic_jacobians; /* 1 = analytic ARAP/depth Jacobians (GPU default); 0 = g2o numeric central differences (delta 1e-9) */
    int32_t verbose;
} deftri_lm_params;

#define DEFTRI_MAX_REPORT_ITERS 1024

typedef struct deftri_report {
    int32_t status;                  /* DEFTRI_STATUS_* */
    int32_t iterations;              /* completed optimize() iterations */
    int32_t trials_total;            /* LM trials (accepted + rejected) */
    int32_t trials_rejected;
    double  chi2_initial;            /* activeRobustChi2 before the first iteration */
    double  chi2_final;
    double  lambda_final;
    double  chi2_iter[DEFTRI_MAX_REPORT_ITERS];   /* accepted chi2 after each iteration */
    int32_t trials_iter[DEFTRI_MAX_REPORT_ITERS]; /* trials used by each iteration */
    /* timing (ms, device-timed with HIP events) */
    double  ms_total;
    double  ms_linearize;            /* residuals + Jacobians + H/b assembly */
    double  ms_factor;               /* multifrontal LDL^T numeric factorization */
    double  ms_solve;                /* forward/backward substitution */
    double  ms_update;               /* oplus + chi2 re-evaluation; the three are -1 (not measured) for
                                        sequential trials unless DEFTRI_TRIAL_EVENTS=1 and on the iterative
                                        plan (per-trial events cost ~6 us of stream time each) */
    /* sizes of the sparse factorization */
    int64_t n_unknowns;
    int64_t nnz_factor;              /* entries of L (incl. dense fronts' boundary rows) */
    double  factor_flops;            /* per factorization */
    int32_t n_fronts;
    int32_t n_levels;
    /* speculative lambda lanes: trials_executed >= trials_total counts the lane trials run,
       including those past the accepted one (their results are discarded) */
    int32_t lanes;
    int32_t trials_executed;
    /* point-sharded solves (deftri_dist_*): this rank, the rank count, the factorization flops of
       all ranks (factor_flops and nnz_factor above are this rank's fronts) */
    int32_t rank;
    int32_t nranks;
    double  factor_flops_total;
    /* uploads on this context that found the same structure (index arrays and counts) as the
       analysed plan and only copied the values (no ordering / symbolic analysis / plan upload) */
    int64_t plan_reuses;
    /* PCG steps (deftri_set_linear_solver): trials solved by PCG, their CG iterations, trials that
       fell back to the factorization, and the device time of the PCG solves (ms, host-timed around
       the solve's final synchronization) */
    int32_t pcg_trials;
    int32_t pcg_fallbacks;           /* multifrontal plan: trials solved by the LDL^T instead; iterative
                                        plan: trials whose PCG failed (rejected, as a failed g2o solve) */
    int64_t pcg_iterations;
    double  ms_pcg;
    /* round 3 */
    int32_t pcg_given_up;            /* multifrontal plan: 1 when two consecutive fallbacks sent the rest of
                                        the call's trials straight to the LDL^T */
    int32_t plan;                    /* DEFTRI_PLAN_MULTIFRONTAL / DEFTRI_PLAN_ITERATIVE */
    /* round 4 (ABI 6) */
    int32_t pcg_continuations;       /* iterative plan: trials whose PCG outran the CG iterations queued
                                        before the evaluation (the last converged count + a margin):
                                        evaluated, restored, continued in chunks of 4 */
} deftri_report;

/* ---- context ---------------------------------------------------------------------- */
/* device >= 0: HIP device ordinal.  device < 0: host-only context (graph construction and
   symbolic analysis only; every device entry point then returns DEFTRI_E_NODEVICE). */
int deftri_ctx_create(int32_t device, deftri_ctx **out);
int deftri_ctx_destroy(deftri_ctx *ctx);
const char *deftri_last_error(const deftri_ctx *ctx);
int deftri_abi_version(void);

/* ---- flat-graph API ---------------------------------------------------------------- */
/* Validate, order (nested dissection), analyse (multifrontal symbolic) and copy to HBM.  A problem
   with the same structure (counts and index arrays) as the one uploaded before keeps the plan and
   the device buffers: only the values are copied (deftri_report.plan_reuses counts these). */
int deftri_problem_upload(deftri_ctx *ctx, const deftri_problem_desc *desc);
/* Run g2o-semantics Levenberg–Marquardt on the device. */
int deftri_solve_lm(deftri_ctx *ctx, const deftri_lm_params *params, deftri_report *report);
/* Speculative lambda lanes (0 = default: env DEFTRI_LM_LANES, else 2 below 3e10 flops per
   factorization (latency-bound) and 1 above; 1 = strictly sequential
   trials; at most 8).  g2o's trials within an iteration use a lambda sequence fixed in advance
   (reject: lambda *= ni, ni *= 2), so up to `lanes` consecutive trials are factored and solved in
   one batched pass (the lane is the second grid dimension of every factor/solve launch), each in
   its own arena and scratch state, and the accept/reject decisions are replayed in trial order:
   results are bit-identical to lanes = 1.  Fewer lanes are used when their buffers would not fit
   in half of the free device memory.  Pays off when the factorization is latency-bound (1k-30k
   correspondences: 11-24% per iteration); at C2 a 3-lane round costs 2.1 trials. */
int deftri_set_lm_lanes(deftri_ctx *ctx, int32_t lanes);
/* Jacobians used by deftri_arap_optimization: 0 (default) g2o's numeric central differences
   (delta 1e-9) for the ARAP and depth edges, as the reference (EdgeARAP has no linearizeOplus,
   g2oTypes.h:341; its analytic one is commented out, g2oTypes.cc:308-331); 1 the closed-form
   Jacobians (an opt-in speed-up, not the reference's arithmetic). */
int deftri_set_jacobian_mode(deftri_ctx *ctx, int32_t analytic);
/* Arithmetic of the factorization's trailing (Schur-complement) updates: 0 (default) fp64
   v_mfma_f64_16x16x4, the reference's precision (SimplicialLDLT in double); 1 fp32 products on
   v_mfma_f32_16x16x4 (operands rounded to fp32, fp32 accumulation per update launch, the result
   subtracted from the fp64 front), the panel factorizations, TRSM and substitution staying fp64.
   For the fp32-vs-fp64 sweep of BASELINE config C5 (tests/test_precision_sweep.py);
   not the reference's arithmetic. */
int deftri_set_factor_precision(deftri_ctx *ctx, int32_t fp32_updates);
/* Linear solver of the LM step (H + lambda I) dx = b inside deftri_solve_lm /
   deftri_arap_optimization (the reference: g2o BlockSolver + LinearSolverEigen, an exact sparse
   LDL^T).  DEFTRI_SOLVER_PCG (default): conjugate gradients preconditioned by the vertex blocks of
   H + lambda I (6x6 T_g, 1x1 scale, 3x3 point), stopped when the CG recurrence's residual r_k
   (not a recomputed b - A dx) satisfies ||r_k|| <= tol ||b|| (tol <= 0: 1e-12); the true residual
   differs from r_k by rounding drift, which tests/test_full_size_props.py measures through
   deftri_eval_hessian_product (< 1e-11 relative at C2).  What a solve that misses its budget or
   breaks down does depends on the plan: the multifrontal plan hands it to its LDL^T (max_iterations
   <= 0: a budget of about one factorization's cost, from the plan's sizes: ~70 at 100k
   correspondences, ~25 for a few hundred points); the iterative plan has no factorization, and the
   trial counts as a failed linear solve — g2o's rejected trial (lambda *= ni) — with a budget of
   1000 iterations when max_iterations <= 0 (DEFTRI_PLAN_ITERATIVE below).  Point-sharded contexts
   take PCG steps on the iterative plan by default and LDL^T steps on the sharded multifrontal plan
   with DEFTRI_SOLVER_DIRECT.  DEFTRI_SOLVER_DIRECT: the multifrontal LDL^T for every trial. */
#define DEFTRI_SOLVER_DIRECT 0
#define DEFTRI_SOLVER_PCG    1
int deftri_set_linear_solver(deftri_ctx *ctx, int32_t solver, double tol, int32_t max_iterations);
/* The last PCG step of this context (solve_lm trial or eval_damped_solve): CG iterations and
   whether it converged (0: the LDL^T solved that step). */
int deftri_last_step_info(const deftri_ctx *ctx, int32_t *pcg_iterations, int32_t *pcg_converged);

/* ---- plan kind (round 3) ---------------------------------------------------------------------
   DEFTRI_PLAN_MULTIFRONTAL: nested dissection + multifrontal LDL^T analysis at upload; PCG steps use
   the sliced matrix-free product where it fits (one KF pair) with the LDL^T as fallback.
   DEFTRI_PLAN_ITERATIVE: the point-sharded matrix-free PCG plan (csrc/spcg.h) — no factorization:
   rows = points grouped by mesh vertex in Morton order, dealt to the ranks in contiguous
   work-balanced ranges; per CG iteration an edge-parallel pass s_e = W_e J_e p over the rank's local
   ARAP edges and a row-parallel gather q_v = sum J_{e,v}^T s_e (+ the folded reprojection / depth
   blocks); sharded: one halo exchange of the boundary rows' (z, p) and ONE all-reduce per CG
   iteration (Chronopoulos-Gear single-reduction CG: r.z, r.r, z.Az and the global-vertex partials
   of A z travel together; plan_info.cg_collectives = 1).  A step whose PCG does not converge within
   the budget (deftri_set_linear_solver max_iterations; <= 0: 1000) counts as a failed linear solve
   (g2o: the trial is rejected; no LDL^T stands behind it).  One rank from 50,000 unknowns: two
   launches per CG iteration (the merged chain), whose alpha is handed from phase 2's workgroup 0 to
   the others through a published value and a flag; this relies on the dispatcher starting a
   launch's workgroups in index order (workgroup 0 resident while the others poll), which HIP does not
   promise: the poll is bounded, and a timeout fails the call with DEFTRI_E_HIP (never a rejected
   trial) and switches the context to a separate alpha launch for later calls.  Any keyframe count (all-pairs graphs, BASELINE C3-C5).
   DEFTRI_PLAN_AUTO (default): ITERATIVE when the step solver is DEFTRI_SOLVER_PCG at upload and the
   context is point-sharded (nranks > 1) or the problem has >= 50,000 unknowns (measured faster from
   C2 up); MULTIFRONTAL otherwise.  Applies to the next deftri_problem_upload.  A
   context on the iterative plan that is asked for what only the factorization has (LDL^T steps or
   solves after deftri_set_linear_solver(DIRECT)) analyses and uploads the multifrontal plan at that
   point, continuing from its current state; deftri_eval_hessian_product stays on the iterative plan
   (its own matrix-free product, H never assembled). */
#define DEFTRI_PLAN_AUTO          0
#define DEFTRI_PLAN_MULTIFRONTAL  1
#define DEFTRI_PLAN_ITERATIVE     2
int deftri_set_plan(deftri_ctx *ctx, int32_t plan);
/* Storage of the ARAP Jacobians the iterative plan's product reads: 0 (default) fp64, 1 fp32 (the
   C5 precision sweep: the product then applies the fp32-rounded J; b, the preconditioner, the
   vectors and every reduction stay fp64).  Applies to the next deftri_problem_upload. */
int deftri_set_jacobian_storage(deftri_ctx *ctx, int32_t fp32);
typedef struct deftri_plan_info {
    int32_t plan;              /* DEFTRI_PLAN_MULTIFRONTAL / DEFTRI_PLAN_ITERATIVE of the uploaded problem */
    int32_t rank, nranks;
    int32_t own_rows;          /* iterative: point rows this rank owns */
    int64_t halo_rows;         /* iterative: rows received from other ranks per exchange */
    int64_t local_arap_edges;  /* iterative: ARAP edges this rank evaluates (owned + halo-only) */
    int64_t n_unknowns;
    int32_t phase1_blocks, row_blocks;
    double  product_bytes;     /* algorithmic bytes of one matrix-free product on this rank */
    int32_t jacobian_fp32;
    int32_t cg_launches;       /* iterative: kernel launches per CG iteration (one rank from 50,000
                                  unknowns: 2, the merged chain — phase 1 forms p.Ap, phase 2 the
                                  update; one rank below that: 3, the dots and the heavy-vertex finish
                                  in last workgroups; sharded: 3, the single-reduction chain —
                                  phase 1 and phase 2 form w = A z, k_sp_update_sd the update) */
    int32_t cg_collectives;    /* iterative: all-reduces per CG iteration (one rank 0; sharded 1, plus
                                  one grouped halo send / receive) */
    int32_t sharded;           /* iterative: the sharded control flow (nranks > 1, or one rank with an
                                  RCCL communicator: deftri_dist_init_rccl(ctx, 1, 0, id)) */
    double  survey_bytes;      /* SURVEY.md §8(d)'s B_pcg of this rank's share: 176 E + 48 R + 40 D + 156 P
                                  (owned ARAP edges, own rows' reprojection / depth edges, own rows) */
    int32_t tiles;             /* iterative: the fused product's tiles (every ARAP edge read once per CG
                                  iteration) — one rank (one keyframe pair since round 5, several since
                                  round 6) or a sharded one-pair plan; 0: the two-phase product */
    int32_t halo_overlap;      /* iterative, sharded (round 5): 1 when the boundary rows' exchange runs
                                  on its own stream beside the interior edges' product */
} deftri_plan_info;
int deftri_get_plan_info(const deftri_ctx *ctx, deftri_plan_info *info);
/* TEST ONLY (no GPU): host emulation of one product q = (H + lambda I) p with the iterative plan's
   decomposition on this rank (deftri_dist_set_transport: rank / nranks and the callback): the rank
   reads only its own rows of p, receives its halo rows through the callback's send / receive in the
   device exchange's global order, all-reduces the global vertices' partials of its owned edges
   (sum), and sums its rows' incidences.  H = sum_e J_e^T W_e J_e over the edges of `desc` with the
   caller's per-edge Jacobians (jarap [E*18] as g2o orders an ARAP edge's vertices, jrep [R*6] 2x3,
   jdep [D*4] point + scale) and scalar weights.  p, q [n], vertex order [T_g][scales][points]; q
   receives this rank's point rows and the global vertices, zeros elsewhere.  stats (may be NULL):
   own rows, halo rows, local ARAP edges, owned ARAP edges. */
int deftri_debug_sp_product(deftri_ctx *ctx, const deftri_problem_desc *desc, const double *jarap, const double *warap,
                            const double *jrep, const double *wrep, const double *jdep, const double *wdep,
                            double lambda, const double *p, double *q, int64_t n, int64_t *stats);
/* ---- simulated observations (upstream producer, host) --------------------------------------
   SLAM::setCameraPoses + getSimulatedDepthMeasurements + createKeyPoints (Modules/System/SLAM.cc:
   223-338): T1w = (I, c1), T2w = (lookAt(c2, moved[0]), c2) as Sophus SE3f (pose = the fp32 unit
   quaternion qx qy qz qw + t); depth_k = z_c * depth_scale_k + N(0, depth_error_mm / 1000) and
   keypoints = KB8 project + N(0, rep_error) rounded to `decimals`, from libstdc++'s
   std::default_random_engine + std::normal_distribution<float> (one fresh engine per function, as
   the reference).  orig / moved [n*3], uv [n*2], depth [n]. */
int deftri_sim_two_view(int32_t n, const float *orig, const float *moved, const float c1[3], const float c2[3],
                        const float kb8_1[8], const float kb8_2[8], float rep_error, int32_t decimals,
                        float depth_error_mm, float depth_scale_1, float depth_scale_2, float *uv1, float *uv2,
                        float *depth1, float *depth2, float pose1[7], float pose2[7]);
/* n draws of one fresh std::default_random_engine + std::normal_distribution<float>(mean, stddev). */
int deftri_sim_normal_stream(int64_t n, float mean, float stddev, float *out);

/* ---- point-sharded ARAP solve (multi-GPU) -------------------------------------------------
   One context per GPU, rank `rank` of `nranks`; every rank uploads the same full problem.  The
   nested-dissection tree is split by rank ranges (a rank owns one subtree, the leading ranks of
   each range also the separator fronts above it); each rank linearizes the edges whose
   first-eliminated vertex it owns, assembles and factors its fronts, and per LM trial sends one
   packed contribution block (lower triangle) up to the owner of its top front's parent, one
   forward-update vector up and receives the boundary solution back; chi2, dx.(lambda dx + b) and
   the zero-pivot flags are all-reduced (sum), the lambda init takes the max of the all-reduced
   diagonal.  Every rank then holds the solution of its own vertices and of its top front's
   boundary vertices (deftri_dist_vertex_owner tells which rank is authoritative for each vertex).
   Transport: RCCL (ncclCommInitRank from a deftri_rccl_unique_id shared by the caller; send/recv
   and all-reduce on the solver stream, over xGMI) or a caller callback through host memory (tests:
   gloo).  Set before deftri_problem_upload / deftri_problem_analyse (it discards the uploaded
   problem); nranks == 1 restores the single-GPU plan.  Diagnostics entry points other than
   deftri_eval_chi2 refuse a sharded context.
   Callback: op 0 all-reduce sum / 1 all-reduce max of n doubles in place (peer = -1), 2 send n
   doubles to `peer`, 3 receive n doubles from `peer`; returns 0 on success.  Every rank makes the
   calls in the same global order. */
typedef int (*deftri_xfer_fn)(void *user, int32_t op, int32_t peer, double *buf, int64_t n);
int deftri_dist_init_rccl(deftri_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t id[128]);
int deftri_dist_set_transport(deftri_ctx *ctx, int32_t nranks, int32_t rank, deftri_xfer_fn fn, void *user);
/* Elimination order of the analysed plan: order[k] = vertex [T_g per pair][scales][points]
   eliminated k-th (nv entries). */
int deftri_plan_vertex_order(const deftri_ctx *ctx, int64_t *order, int64_t nv);
/* Owning rank of every vertex [T_g per pair][scales][points] of the analysed problem (nv entries). */
int deftri_dist_vertex_owner(const deftri_ctx *ctx, int32_t *owner, int64_t nv);
/* 0/1 per edge of the analysed problem: edges this rank linearizes (any output may be NULL). */
int deftri_dist_owned_edges(const deftri_ctx *ctx, uint8_t *rep, uint8_t *dep, uint8_t *arap);
/* TEST ONLY: host emulation of this rank's damped solve (H_q + lambda on its diagonal) x = b_q, with
   H_q, b_q this rank's partial system (row-major n x n, the sum over ranks is H, b), exchanging
   through the callback transport; x receives the solution of the rank's own and boundary dofs. */
int deftri_debug_plan_solve_dist(deftri_ctx *ctx, const double *Hq, double lambda, const double *bq, double *x,
                                 int64_t n);

/* Copy the current state back: points [P*3], scales [S], tg [Q*7] (any may be NULL). */
int deftri_download(deftri_ctx *ctx, double *points, double *scales, double *tg);
/* Reset the device state to the uploaded initial values (no re-analysis). */
int deftri_reset_state(deftri_ctx *ctx);

/* ---- diagnostics (parity tests) ----------------------------------------------------- */
/* activeRobustChi2 at the current device state. */
int deftri_eval_chi2(deftri_ctx *ctx, double *chi2);
/* Linearize at the current state and return b (gradient side, g2o sign: b = -J^T W e)
   in the vertex order [T_g(6) per pair][scales][points(3)], and the diagonal of H. */
int deftri_eval_gradient(deftri_ctx *ctx, double *b, double *hdiag, int64_t n);
/* y = H x for the current linearization (same vertex order).  On the iterative plan: the CG
   chain's own matrix-free product kernels (H is never assembled; analytic-Jacobian linearization,
   as deftri_eval_damped_solve), so a solve's true residual ||b - (H + lambda I) x|| can be measured
   at any size; on the multifrontal plan: the assembled blocks. */
int deftri_eval_hessian_product(deftri_ctx *ctx, const double *x, double *y, int64_t n);
/* Solve (H + lambda I) x = rhs (analytic-Jacobian linearization at the current state) with the
   configured step solver (deftri_set_linear_solver: PCG with LDL^T fallback, or the LDL^T). */
int deftri_eval_damped_solve(deftri_ctx *ctx, double lambda, const double *rhs, double *x, int64_t n);
/* Number of unknowns of the uploaded problem. */
int64_t deftri_num_unknowns(const deftri_ctx *ctx);

/* Validate + analyse (ordering, multifrontal plan) without touching a device. */
int deftri_problem_analyse(deftri_ctx *ctx, const deftri_problem_desc *desc);
/* Plan statistics of the analysed problem: n_unknowns, nnz_factor, factor_flops, n_fronts,
   n_levels (other report fields zero). */
int deftri_plan_stats(const deftri_ctx *ctx, deftri_report *report);
/* TEST ONLY: execute the analysed multifrontal plan with host loops on a dense, row-major
   n x n H (vertex order as above) to check the symbolic analysis without a GPU.  Not used by
   any solve path. */
int deftri_debug_plan_solve(deftri_ctx *ctx, const double *H, double lambda, const double *rhs,
                            double *x, int64_t n);
/* Per-kernel device timing of one LM trial (linearize + assemble + setLambda + LDL^T + solve),
   each launch bracketed by HIP events on the solver's stream.  flops are algorithmic counts
   for the dense factor kernels (0 where not defined). */
typedef struct deftri_kernel_stat {
    char    name[32];
    int64_t launches;
    double  ms;          /* summed device time */
    double  flops;       /* algorithmic flops of all launches */
    double  bytes;       /* algorithmic HBM bytes of all launches (0 where not defined) */
} deftri_kernel_stat;
int deftri_profile_trial(deftri_ctx *ctx, double lambda, deftri_kernel_stat *stats,
                         int32_t max_stats, int32_t *n_stats);

/* sizeof() of the ABI structs for binding checks: 0 deftri_problem_desc, 1 deftri_lm_params,
   2 deftri_report, 3 deftri_keyframe, 4 deftri_map, 5 deftri_ba_desc, 6 deftri_pixels_error,
   7 deftri_plan_info, 8 deftri_deformation_params, 9 deftri_deformation_report,
   10 deftri_deformation_eval. */
int64_t deftri_sizeof(int32_t which);

/* ---- map-level API (Modules/Optimization/g2oBundleAdjustment.h:56-60) ---------------- */
/* A keyframe as the solver reads/writes it (Modules/Map/KeyFrame.h): slots i = 0..n_slots-1
   hold an optional MapPoint (point_id < 0 = null), its keypoint, octave and simulated depth. */
typedef struct deftri_keyframe {
    int64_t id;                 /* KeyFrame id */
    double  pose[7];            /* T_cw as qx qy qz qw tx ty tz (from Sophus::SE3f) */
    float   kb8[8];             /* calibration */
    int32_t n_scales;           /* octave table size */
    const float *inv_sigma2;    /* [n_scales] Frame::vInvSigma2_ (Frame.cc:61-75) */
    double  depth_scale;        /* estimatedDepthScale_ (in/out) */
    int32_t n_slots;
    int64_t *point_id;          /* [n_slots] MapPoint id, < 0 = null slot                  */
    float   *point_pos;         /* [n_slots*3] MapPoint world position (in/out, fp32 as the reference) */
    const int32_t *obs_index;   /* [n_slots] Map::isMapPointInKeyFrame(point, kf) (< 0 = none) */
    const float *kp_uv;         /* [n_obs*2] keypoints by observation index */
    const int32_t *kp_octave;   /* [n_obs] */
    const float *depth;         /* [n_obs] simulated depth per observation index (KeyFrame.cc:123-125) */
    int32_t n_obs;
} deftri_keyframe;

/* One entry of Map::mGTransformation_ (Modules/Map/Map.cc:323-343): the transformation stored for
   the ordered KeyFrame-id pair (kf1, kf2).  insertGlobalKeyFramesTransformation stores T for
   (kf1, kf2) and T.inverse() (Sophus, fp32) for (kf2, kf1): pass both entries. */
typedef struct deftri_global_entry {
    int64_t kf1, kf2;
    double  t[7];                 /* qx qy qz qw tx ty tz */
} deftri_global_entry;

typedef struct deftri_map {
    int32_t n_keyframes;
    deftri_keyframe *keyframes;   /* in the reference's unordered_map iteration order */
    double global_t[7];           /* out: the optimized T_g, stored by the reference as (0, 1) (:1007).
                                     in (legacy, only when n_global == 0): T for the first pair */
    int32_t n_global;             /* in: entries of the map's global-transformation table */
    const deftri_global_entry *globals;   /* every pair (kf1, kf2) of the graph starts from
                                     getGlobalKeyFramesTransformation(kf1.id, kf2.id) (:664): the
                                     entry for that ordered id pair, identity when absent */
} deftri_map;

/* arapOptimization(Map*, rep, global, arap, alpha, beta, depthError, nIt, optimizationUpdate)
   (g2oBundleAdjustment.cc:608).  Builds the graph on the host (Delaunay mesh, cotangent
   weights, per-vertex R_i, reference indexing), solves on the device, writes back
   positions (fp32), depth scales and the global transformation.  optimization_update may be
   NULL; when given it receives sum ||p_old - p_new|| (:974-990). */
int deftri_arap_optimization(deftri_ctx *ctx, deftri_map *map, double rep_weight,
                             double global_weight, double arap_weight, double alpha,
                             double beta, float depth_error, int32_t n_iterations,
                             double *optimization_update, deftri_report *report);

/* PixelsError (Modules/Utils/CommonTypes.h:23-30). */
typedef struct deftri_pixels_error {
    double avgc1, avgc2, avg;      /* mean |obs - proj| per camera (last pair), their average */
    double desvc1, desvc2, desv;   /* RMS |obs - proj| per camera (last pair), their average */
} deftri_pixels_error;

/* calculatePixelsStandDev(Map, PixelsError&) (Modules/Utils/Geometry.cc:370-498) on the device:
   for every keyframe pair (k1, k2 > k1 in map order; camera 1 = k2, camera 2 = k1) and every slot
   whose MapPoints both exist and are observed, the fp32 homogeneous projection error; per pair the
   reference's formulas (nMatches and the mean accumulators carry across pairs, the squared sums
   do not; the values of the last pair are returned).  Reads the map's fp32 positions. */
int deftri_pixels_stand_dev(deftri_ctx *ctx, const deftri_map *map, deftri_pixels_error *out);

/* ---- map-error measurements (Modules/Utils/Measurements.cc) --------------------------------- */
/* measureSimAbsoluteMapErrors (:8-98): MapPoints 2j and 2j+1 (by id) against original[j] / moved[j]
   for j < (#MapPoints)/2; the figures the reference prints / writes to Experiment.txt, in mm. */
typedef struct deftri_abs_errors {
    double average_movement;        /* mean |original - moved| */
    double average_error_original;  /* mean |p_2j - original| */
    double average_error_moved;     /* mean |p_2j+1 - moved| */
    double average_error;           /* (sum of both) / #MapPoints ("Av. error") */
    double rmse;                    /* sqrt(sum of squared errors / #MapPoints) ("RMSE") */
    int64_t point_count;            /* #MapPoints */
} deftri_abs_errors;
int deftri_measure_sim_absolute_map_errors(int32_t device, const deftri_map *map, int32_t n_points,
                                           const float *original, const float *moved, deftri_abs_errors *out);
/* measureRelativeMapErrors (:350-518), per keyframe pair in the map's order: the values after that
   pair (the accumulators carry over pairs, as in the reference).  Depth uses the per-index simulated
   measurement (the reference's depth-image lookup throws in the simulation). */
typedef struct deftri_rel_errors {
    int64_t kf1, kf2;               /* KeyFrame ids (k2->first, k1->first) */
    int32_t reported;               /* validPairs > 1: the reference prints / writes the pair */
    double rel_error;               /* sum ||(pi2 - pj2) - (pi1 - pj1)||^2 / mesh area ("Rel. error") */
    double depth_error;             /* sum (d - z s)^2 ("depthError") */
    double global_t_error;          /* sum ||(R pi2 - t - pi1) + (R pj2 - t - pj1)||^2 / area */
    double area;                    /* the pair's mesh surface area */
    int64_t valid_pairs, n_matches;
} deftri_rel_errors;
int deftri_measure_relative_map_errors(int32_t device, const deftri_map *map, deftri_rel_errors *out,
                                       int32_t max_pairs, int32_t *n_pairs);


/* Mapping::triangulateSimulatedMapPoints (Modules/Mapping/Mapping.cc:280-349) for Triangulation.method
   "NRSLAM", seed.location "FarPoints" (Simulation.yaml): per correspondence i, KB8 unproject of
   uv1[i] / uv2[i] (KannalaBrandt8.cc:51-83), triangulateNRSLAM (Geometry.cc:103-153) and
   isValidParallax (Mapping.cc:351-366: both depths >= 0, cos parallax <= min_cos).  Poses are
   T_cw as 3x4 fp32 row-major [R | t] (Sophus::SE3f::matrix3x4()).  Outputs: world points for KF 1
   and KF 2 [n*3] and valid[n] (the reference's `continue` skips invalid ones). */
int deftri_triangulate_nrslam(deftri_ctx *ctx, int32_t n, const float *uv1, const float *uv2,
                              const float *kb8_1, const float *kb8_2, const float *T1w, const float *T2w,
                              float min_cos, float *x3d_1, float *x3d_2, uint8_t *valid);

/* Build the flattened graph only (no solve): the arrays are owned by the context and stay
   valid until the next call on it.  Used by the parity tests to compare indexing. */
/* MapPoint id of every point vertex of the last graph deftri_arap_build_graph built (n = its
   n_points): the write-back key of :974-990. */
int deftri_arap_graph_point_ids(const deftri_ctx *ctx, int64_t *ids, int64_t n);
/* Graph builds of this context so far answered by the memo (the same map: NLopt's clones) and by
   the structure memo (deformationOptimization's next round: positions, depth scales and T_g moved,
   every pair's Delaunay triangulation still valid — the values refreshed in place, the descriptor
   equal bit for bit to a full build's), and the host time of the last build in ms. */
int deftri_graph_stats(const deftri_ctx *ctx, int64_t *memo_hits, int64_t *struct_hits, double *ms_last);
/* Full graph builds' keyframe meshes that were repaired from the previous build's triangulation of
   the same vertices (Lawson flips with exact predicates, then the same strict uniqueness check as the
   structure memo — so the mesh equals a new Delaunay triangulation triangle for triangle) instead of
   triangulated anew, and the flips they took, over this context's life. */
int deftri_graph_repairs(const deftri_ctx *ctx, int64_t *meshes, int64_t *flips);
/* Keyframe pairs of the graphs this context builds (deftri_arap_build_graph / _optimization): 0
   (default) every pair (a, b > a) in map order, as the reference's loop (g2oBundleAdjustment.cc:
   640-645); w > 0 only pairs with b - a <= w (a sliding window: the documented deviation used for
   BASELINE C5's 20 keyframes, 19 consecutive pairs at w = 1). */
int deftri_set_pair_window(deftri_ctx *ctx, int32_t window);
int deftri_arap_build_graph(deftri_ctx *ctx, const deftri_map *map, double rep_weight,
                            double arap_weight, float depth_error,
                            const deftri_problem_desc **desc_out);

/* ---- deformationOptimization (g2oBundleAdjustment.cc:446-606), round 5 --------------------
   The outer loop in native code: rounds i = 1 .. n_optimizations while the last round's update
   sum ||p_old - p_new|| >= 1e-4 n_map_points (:482).  A round of selection 0 ("g2oArap") is one
   arapOptimization with the current weights; selection 1 ("twoOptimizations" + weightsSelection
   "nlopt", the Simulation.yaml default) first runs NLopt's LN_NELDERMEAD over (rep, global, arap)
   within [lb, ub] (xtol_rel, xtol_abs, maxeval; :486-530) — NLopt 2.x's nldrmd.c with its default
   initial step, elimdim and relstop restated (deftri/nlopt_nm.py is the same algorithm) — whose
   every evaluation is outerObjective (nloptOptimization.cc:4-37): arapOptimization on a clone of
   a clone of the map as the round started (:499, nloptOptimization.cc:13; Map::clone, Map.cc:30-58:
   here a copy of the positions and depth scales, the rest shared read-only — with the reference's
   two observable properties: the clone's global table is EMPTY, Map::clone does not copy
   mGTransformation_, so its pairs start T_g at the identity; and the clone iterates its keyframes
   in the order deftri_keyframe_order gives), then calculatePixelsStandDev
   on the device, f = log(desvc1)^2 + log(desvc2)^2; then arapOptimization on the map itself with
   the optimum, whose weights the next round starts from.  A search that ends on a failure code
   (nldrmd's degenerate initial simplex) returns DEFTRI_E_SEARCH before that round's
   arapOptimization (the reference's nlopt::opt::optimize throws there); weightsSelection "eigen"
   is selection 0: the reference's Eigen::LevenbergMarquardt::minimize returns
   ImproperInputParameters before evaluating anything (its functor declares 2 values for 3 inputs,
   m < n, EigenOptimization.h:31, g2oBundleAdjustment.cc:532-550) and the round runs
   arapOptimization with the unchanged weights.  The map's positions and depth scales are
   written back in place after every round and global_t holds the last T_g; the global table the
   next round reads is updated as Map::insertGlobalKeyFramesTransformation(0, 1, T) does
   (Map.cc:323-330: T and its fp32 inverse).  The Eigen-LM weight search (weightsSelection
   "eigen", EigenOptimization.h) is not built (its functor reads 3 of 2 declared inputs). */
typedef struct deftri_deformation_params {
    int32_t selection;            /* 0 g2oArap (fixed weights), 1 twoOptimizations + nlopt */
    double  rep, global, arap;    /* Optimization.* weights: the search's start */
    double  alpha, beta;          /* stored on the ARAP edges, unused by their error (as the reference) */
    float   depth_error;          /* sigma_d (m) */
    int32_t n_iterations;         /* LM iterations per arapOptimization (Optimization.numberOfIterations) */
    int32_t n_optimizations;      /* outer rounds at most (Optimization.numberOfOptimizations) */
    double  lb[3], ub[3];         /* nlopt bounds of (rep, global, arap) */
    double  xtol_rel, xtol_abs;   /* nlopt.relTolerance / absTolerance */
    int32_t maxeval;              /* nlopt.numberOfIterations */
    int32_t n_map_points;         /* |MapPoints| of the map (the stop test's scale) */
} deftri_deformation_params;
typedef struct deftri_deformation_eval {
    int32_t round, eval;          /* 1-based round, 1-based evaluation inside the round's search */
    double  x[3], f;              /* the weights evaluated and outerObjective's value */
} deftri_deformation_eval;
typedef struct deftri_deformation_report {
    int32_t rounds;               /* outer rounds run */
    int32_t arap_calls;           /* arapOptimization calls (evaluations + one per round) */
    double  weights[3];           /* the last round's weights */
    double  minf;                 /* the last search's best objective */
    int32_t nlopt_result;         /* the last search's result code (1 success, 4 xtol, 5 maxeval, -1 failure) */
    double  update;               /* the last round's update */
    double  seconds;              /* wall time of the call */
    deftri_deformation_eval *evals;   /* caller's buffer (may be NULL): every evaluation, in order */
    int32_t max_evals, n_evals;   /* its capacity; evaluations recorded (all, up to the capacity) */
    double  round_update[64];     /* per round (first 64): its update, */
    double  round_weights[64][3]; /* its weights */
} deftri_deformation_report;
int deftri_deformation_optimization(deftri_ctx *ctx, deftri_map *map, const deftri_deformation_params *params,
                                    deftri_deformation_report *report);
/* Map::insertGlobalKeyFramesTransformation(0, 1, T) of the map-level call's T_g (global_t):
   the (kf1, kf2) entry and its fp32 inverse for (kf2, kf1), each as the g2o::SE3Quat the next
   arapOptimization reads back (getGlobalKeyFramesTransformation, :664) — Sophus SE3f from the
   estimate cast to float (quaternion normalized in float), the inverse as the conjugate rotation and
   -(R^T t) by Eigen's quaternion-vector product, in float.  The one implementation the native outer
   loop and the host mirror's Map model both use.  No context, no GPU. */
int deftri_global_insert(const double t7[7], double fwd7[7], double inv7[7]);
/* The KeyFrame iteration order of Map::mKeyFrames_ (std::unordered_map<ID, KeyFrame_>, Map.h:185),
   which every reference loop over keyframes follows (:640-645, Geometry.cc:387): `insert_ids` in the
   order Map::insertKeyFrame was called; `clones` applications of Map::clone (Map.cc:30-58, which
   re-inserts the keyframes in the source's iteration order) after that.  Evaluated with the same
   standard-library container (libstdc++), not restated.  out[n]: ids in iteration order.  No GPU. */
int deftri_keyframe_order(const int64_t *insert_ids, int32_t n, int32_t clones, int64_t *out);
/* TEST ONLY (no GPU): the restated NLopt LN_NELDERMEAD on a caller objective f(x, n, user) over n <= 8
   dimensions — the search deftri_deformation_optimization runs.  x: in the start, out the best;
   *result the NLopt result code (1 success, 4 xtol reached, 5 maxeval reached, -1 failure), *minf,
   *nevals.  Returns 0, or DEFTRI_E_ARG (bad arguments, x0 outside the bounds). */
typedef double (*deftri_objective_fn)(const double *x, int32_t n, void *user);
int deftri_debug_nelder_mead(deftri_objective_fn f, void *user, int32_t n, double *x, const double *lb,
                             const double *ub, double xtol_rel, double xtol_abs, int32_t maxeval, double *minf,
                             int32_t *nevals, int32_t *result);

/* ==== bundle adjustment ============================================
 * The BlockSolver_6_3 Schur LM of the reference's BA entry points:
 *   bundleAdjustment(Map*)             g2oBundleAdjustment.cc:38-138   (optimize(20), KF 0 fixed)
 *   localBundleAdjustment(Map*, ID)    g2oBundleAdjustment.cc:245-444  (optimize(5), outlier
 *                                      levels, robust kernels off, optimize(10))
 *   poseOnlyOptimization(Frame&)       g2oBundleAdjustment.cc:140-243  (4 rounds x optimize(10))
 * Vertices: poses g2o::VertexSE3Expmap (6 dof, T <- exp(d) * T), points VertexSBAPointXYZ
 * (3 dof, marginalized).  Edges: EdgeSE3ProjectXYZ (g2oTypes.h:150-189, linearizeOplus
 * g2oTypes.cc:121-142) with info = invSigma2(octave) * I2 and optional Huber; with every point
 * fixed the edges are EdgeSE3ProjectXYZOnlyPose (g2oTypes.h:191-229, g2oTypes.cc:173-189).
 * On the device: per-edge residual/Jacobian, per-point 3x3 blocks, per-pose 6x6 blocks, the
 * Schur complement S = Hpp - sum_l Hpl Hll^-1 Hlp (dense, 6 x free poses), a dense LDL^T of S,
 * point back-substitution.  Points may be sharded over ranks (one rank per GPU): each rank
 * uploads every pose but only its points and their edges; the pose blocks and S are summed
 * across ranks (RCCL all-reduce, or a caller-provided all-reduce) once per LM trial. */
typedef struct deftri_ba_ctx deftri_ba_ctx;

typedef struct deftri_ba_desc {
    int32_t n_poses;             /* K  VertexSE3Expmap                                      */
    int32_t n_points;            /* P  VertexSBAPointXYZ (marginalized)                      */
    int32_t n_edges;             /* E  EdgeSE3ProjectXYZ                                     */
    int32_t reserved;
    const double  *poses;        /* [K*7] T_cw: qx qy qz qw tx ty tz                         */
    const uint8_t *pose_fixed;   /* [K] 1 = setFixed(true); NULL = none                      */
    const float   *pose_kb8;     /* [K*8] KannalaBrandt8 fx fy cx cy k0..k3 of each pose's KF */
    const double  *points;       /* [P*3] world positions                                   */
    const uint8_t *point_fixed;  /* [P] 1 = constant (poseOnly's Xworld); NULL = none        */
    const int32_t *edge_point;   /* [E] */
    const int32_t *edge_pose;    /* [E] */
    const double  *edge_obs;     /* [E*2] keypoint (u, v)                                   */
    const double  *edge_info;    /* [E]   information = edge_info * I2                      */
    const uint8_t *edge_level;   /* [E] g2o edge level; NULL = all 0                        */
    const uint8_t *edge_robust;  /* [E] 1 = RobustKernelHuber(huber_delta); NULL = all 1     */
    double huber_delta;          /* reference: (float)sqrt(5.99)                            */
} deftri_ba_desc;

/* Caller-supplied all-reduce over ranks (tests, non-RCCL transports): n doubles in HOST memory,
   reduced in place; op 0 = sum, 1 = max.  The library stages the device buffer through host
   memory around the call (the RCCL path reduces device-resident buffers directly).  Returns 0
   on success. */
typedef int (*deftri_allreduce_fn)(void *user, double *host_buf, int64_t n, int32_t op);

int deftri_ba_create(int32_t device, deftri_ba_ctx **out);
int deftri_ba_destroy(deftri_ba_ctx *ctx);
const char *deftri_ba_last_error(const deftri_ba_ctx *ctx);
/* Copy the graph to HBM (edges are kept in point order internally; per-edge in/out arrays of
   this API always use the caller's edge order). */
int deftri_ba_upload(deftri_ba_ctx *ctx, const deftri_ba_desc *desc);
/* vertex->setEstimate(): replace poses [K*7] and/or points [P*3] (NULL = unchanged). */
int deftri_ba_set_state(deftri_ba_ctx *ctx, const double *poses, const double *points);
/* e->setLevel() / e->setRobustKernel(0 or Huber) for every edge (NULL = unchanged). */
int deftri_ba_set_edge_flags(deftri_ba_ctx *ctx, const uint8_t *level, const uint8_t *robust);
/* optimizer.initializeOptimization(level); optimizer.optimize(params->n_iterations).  Active
   edges = level `level` with a non-fixed vertex; active vertices = those with an active edge. */
int deftri_ba_solve_lm(deftri_ba_ctx *ctx, const deftri_lm_params *params, int32_t level,
                       deftri_report *report);
/* e->computeError() on every edge (active or not) whose mask entry is non-zero (caller edge
   order; NULL = every edge). */
int deftri_ba_compute_errors(deftri_ba_ctx *ctx, const uint8_t *mask);
/* Per edge (caller order): e->chi2() of the cached error (no robust kernel) and
   e->isDepthPositive() at the current state.  Either output may be NULL. */
int deftri_ba_edge_chi2(deftri_ba_ctx *ctx, double *chi2, uint8_t *depth_positive);
/* Current estimates: poses [K*7], points [P*3] (either may be NULL). */
int deftri_ba_download(deftri_ba_ctx *ctx, double *poses, double *points);
/* Diagnostics (parity tests): initializeOptimization(level), linearize at the current state and
   form the damped Schur system at `lambda`.  Outputs (any may be NULL): chi2 (activeRobustChi2,
   summed over ranks), S [ns*ns] (row-major, full) and rhs [ns] of the reduced pose system, dx
   [6K + 3P] (poses in pose order, 0 for fixed/inactive; then points), b [6K + 3P] (g2o sign).
   *ns receives 6 x (number of free active poses). */
int deftri_ba_eval_system(deftri_ba_ctx *ctx, int32_t level, double lambda, double *chi2, double *S,
                          double *rhs, double *dx, double *b, int32_t *ns);
/* Point-sharded multi-GPU: this context is rank `rank` of `nranks`.  Either RCCL (the
   production path: ncclCommInitRank over xGMI, all-reduce on the solver stream; the 128-byte id
   comes from deftri_rccl_unique_id on rank 0, shared by the caller) or a caller-supplied
   all-reduce (tests: e.g. gloo through host memory).  nranks == 1 with a NULL id / fn clears the
   setting (an RCCL communicator of one rank is kept when an id is given). */
int deftri_rccl_unique_id(uint8_t id[128]);
int deftri_ba_dist_init_rccl(deftri_ba_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t id[128]);
int deftri_ba_dist_set_allreduce(deftri_ba_ctx *ctx, int32_t nranks, int32_t rank, deftri_allreduce_fn fn,
                                 void *user);
/* Per-kernel device timing of one LM trial of the BA path (HIP events on the solver stream). */
int deftri_ba_profile_trial(deftri_ba_ctx *ctx, double lambda, deftri_kernel_stat *stats, int32_t max_stats,
                            int32_t *n_stats);

#ifdef __cplusplus
}
#endif
#endif /* DEFTRI_H */
