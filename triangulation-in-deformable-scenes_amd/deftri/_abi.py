"""ctypes mirror of include/deftri.h (the C-ABI boundary).

Kept field-for-field identical to the header; tests/test_abi.py checks the struct sizes
against the compiled library (deftri_sizeof_* exports).
"""
import ctypes as C

i32, i64, f32, f64 = C.c_int32, C.c_int64, C.c_float, C.c_double
P = C.POINTER

DEFTRI_OK = 0
DEFTRI_E_ARG = -1
DEFTRI_E_HIP = -2
DEFTRI_E_NOPROBLEM = -3
DEFTRI_E_NUMERIC = -4
DEFTRI_E_NODEVICE = -5
DEFTRI_E_GRAPH = -6
DEFTRI_STATUS_OK = 0
DEFTRI_STATUS_TERMINATE = 1
DEFTRI_SOLVER_DIRECT = 0
DEFTRI_SOLVER_PCG = 1
DEFTRI_PLAN_AUTO = 0
DEFTRI_PLAN_MULTIFRONTAL = 1
DEFTRI_PLAN_ITERATIVE = 2
DEFTRI_MAX_REPORT_ITERS = 1024


class ProblemDesc(C.Structure):
    _fields_ = [
        ("n_points", i32), ("n_pairs", i32), ("n_scales", i32), ("n_cams", i32),
        ("n_rep", i32), ("n_depth", i32), ("n_arap", i32), ("n_rot", i32),
        ("points", P(f64)), ("tg", P(f64)), ("scales", P(f64)),
        ("cam_kb8", P(f32)), ("cam_pose", P(f64)),
        ("rep_point", P(i32)), ("rep_cam", P(i32)), ("rep_obs", P(f64)), ("rep_info", P(f64)),
        ("huber_delta", f64),
        ("dep_point", P(i32)), ("dep_scale", P(i32)), ("dep_cam", P(i32)),
        ("dep_meas", P(f64)), ("dep_info", P(f64)),
        ("arap_pts", P(i32)), ("arap_pair", P(i32)), ("arap_rot", P(i32)), ("arap_w", P(f64)),
        ("rot", P(f64)), ("pair_area", P(f64)), ("pair_info", P(f64)),
        ("order_xy", P(f64)),
    ]


class LMParams(C.Structure):
    _fields_ = [("n_iterations", i32), ("max_trials", i32), ("tau", f64), ("user_lambda", f64),
                ("analytic_jacobians", i32), ("verbose", i32)]


class Report(C.Structure):
    _fields_ = [
        ("status", i32), ("iterations", i32), ("trials_total", i32), ("trials_rejected", i32),
        ("chi2_initial", f64), ("chi2_final", f64), ("lambda_final", f64),
        ("chi2_iter", f64 * DEFTRI_MAX_REPORT_ITERS), ("trials_iter", i32 * DEFTRI_MAX_REPORT_ITERS),
        ("ms_total", f64), ("ms_linearize", f64), ("ms_factor", f64), ("ms_solve", f64),
        ("ms_update", f64),
        ("n_unknowns", i64), ("nnz_factor", i64), ("factor_flops", f64), ("n_fronts", i32),
        ("n_levels", i32), ("lanes", i32), ("trials_executed", i32),
        ("rank", i32), ("nranks", i32), ("factor_flops_total", f64), ("plan_reuses", i64),
        ("pcg_trials", i32), ("pcg_fallbacks", i32), ("pcg_iterations", i64), ("ms_pcg", f64),
        ("pcg_given_up", i32), ("plan", i32), ("pcg_continuations", i32),
    ]

    def as_dict(self):
        it = min(self.iterations, DEFTRI_MAX_REPORT_ITERS)
        return {
            "status": self.status, "iterations": self.iterations,
            "trials_total": self.trials_total, "trials_rejected": self.trials_rejected,
            "chi2_initial": self.chi2_initial, "chi2_final": self.chi2_final,
            "lambda_final": self.lambda_final,
            "chi2_iter": list(self.chi2_iter[:it]), "trials_iter": list(self.trials_iter[:it]),
            "ms_total": self.ms_total, "ms_linearize": self.ms_linearize,
            "ms_factor": self.ms_factor, "ms_solve": self.ms_solve, "ms_update": self.ms_update,
            "n_unknowns": self.n_unknowns, "nnz_factor": self.nnz_factor,
            "factor_flops": self.factor_flops, "n_fronts": self.n_fronts, "n_levels": self.n_levels,
            "lanes": self.lanes, "trials_executed": self.trials_executed,
            "rank": self.rank, "nranks": self.nranks, "factor_flops_total": self.factor_flops_total,
            "plan_reuses": self.plan_reuses,
            "pcg_trials": self.pcg_trials, "pcg_fallbacks": self.pcg_fallbacks,
            "pcg_iterations": self.pcg_iterations, "ms_pcg": self.ms_pcg,
            "pcg_given_up": self.pcg_given_up,
            "pcg_continuations": self.pcg_continuations,
            "plan": {DEFTRI_PLAN_MULTIFRONTAL: "multifrontal", DEFTRI_PLAN_ITERATIVE: "iterative"}.get(self.plan, "none"),
        }


class PixelsError(C.Structure):
    _fields_ = [("avgc1", f64), ("avgc2", f64), ("avg", f64), ("desvc1", f64), ("desvc2", f64), ("desv", f64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class KeyFrameC(C.Structure):
    _fields_ = [
        ("id", i64), ("pose", f64 * 7), ("kb8", f32 * 8), ("n_scales", i32),
        ("inv_sigma2", P(f32)), ("depth_scale", f64), ("n_slots", i32),
        ("point_id", P(i64)), ("point_pos", P(f32)), ("obs_index", P(i32)),
        ("kp_uv", P(f32)), ("kp_octave", P(i32)), ("depth", P(f32)), ("n_obs", i32),
    ]


class GlobalEntryC(C.Structure):
    _fields_ = [("kf1", i64), ("kf2", i64), ("t", f64 * 7)]


class MapC(C.Structure):
    _fields_ = [("n_keyframes", i32), ("keyframes", P(KeyFrameC)), ("global_t", f64 * 7),
                ("n_global", i32), ("globals", P(GlobalEntryC))]


class DeformationParams(C.Structure):
    _fields_ = [("selection", i32), ("rep", f64), ("global_", f64), ("arap", f64), ("alpha", f64), ("beta", f64),
                ("depth_error", f32), ("n_iterations", i32), ("n_optimizations", i32), ("lb", f64 * 3),
                ("ub", f64 * 3), ("xtol_rel", f64), ("xtol_abs", f64), ("maxeval", i32), ("n_map_points", i32)]


class DeformationEval(C.Structure):
    _fields_ = [("round", i32), ("eval", i32), ("x", f64 * 3), ("f", f64)]


class DeformationReport(C.Structure):
    _fields_ = [("rounds", i32), ("arap_calls", i32), ("weights", f64 * 3), ("minf", f64), ("nlopt_result", i32),
                ("update", f64), ("seconds", f64), ("evals", P(DeformationEval)), ("max_evals", i32),
                ("n_evals", i32), ("round_update", f64 * 64), ("round_weights", (f64 * 3) * 64)]


OBJECTIVE_FN = C.CFUNCTYPE(C.c_double, P(C.c_double), C.c_int32, C.c_void_p)


class AbsErrorsC(C.Structure):
    _fields_ = [("average_movement", f64), ("average_error_original", f64), ("average_error_moved", f64),
                ("average_error", f64), ("rmse", f64), ("point_count", i64)]


class RelErrorsC(C.Structure):
    _fields_ = [("kf1", i64), ("kf2", i64), ("reported", i32), ("rel_error", f64), ("depth_error", f64),
                ("global_t_error", f64), ("area", f64), ("valid_pairs", i64), ("n_matches", i64)]


class PlanInfo(C.Structure):
    _fields_ = [("plan", i32), ("rank", i32), ("nranks", i32), ("own_rows", i32), ("halo_rows", i64),
                ("local_arap_edges", i64), ("n_unknowns", i64), ("phase1_blocks", i32), ("row_blocks", i32),
                ("product_bytes", f64), ("jacobian_fp32", i32), ("cg_launches", i32), ("cg_collectives", i32),
                ("sharded", i32), ("survey_bytes", f64), ("tiles", i32), ("halo_overlap", i32)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["plan"] = {DEFTRI_PLAN_MULTIFRONTAL: "multifrontal", DEFTRI_PLAN_ITERATIVE: "iterative"}.get(self.plan, "none")
        return d


class KernelStat(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", i64), ("ms", f64), ("flops", f64), ("bytes", f64)]


class BADesc(C.Structure):
    _fields_ = [
        ("n_poses", i32), ("n_points", i32), ("n_edges", i32), ("reserved", i32),
        ("poses", P(f64)), ("pose_fixed", P(C.c_uint8)), ("pose_kb8", P(f32)),
        ("points", P(f64)), ("point_fixed", P(C.c_uint8)),
        ("edge_point", P(i32)), ("edge_pose", P(i32)), ("edge_obs", P(f64)), ("edge_info", P(f64)),
        ("edge_level", P(C.c_uint8)), ("edge_robust", P(C.c_uint8)),
        ("huber_delta", f64),
    ]


# int (*)(void *user, double *host_buf, int64_t n, int32_t op)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, P(f64), i64, i32)
# int (*)(void *user, int32_t op, int32_t peer, double *buf, int64_t n)   (deftri_xfer_fn)
XFER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, i32, i32, P(f64), i64)


def ptr(a, ctype):
    """Pointer into a contiguous numpy array (None for None)."""
    if a is None:
        return None
    return a.ctypes.data_as(P(ctype))
