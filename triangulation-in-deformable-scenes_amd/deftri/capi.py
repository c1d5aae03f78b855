"""ctypes binding of libdeftri.so (include/deftri.h).

The library is built in-tree (csrc/Makefile -> triangulation-in-deformable-scenes_amd/libdeftri.so).
There is no CPU fallback: if the library is missing, `load()` raises, and every solve entry
point runs on the GPU or returns an error.
"""
import ctypes as C
import time
import os
import pathlib

import numpy as np

from . import _abi
from .problem import Problem

PKG_ROOT = pathlib.Path(__file__).resolve().parent.parent
LIB_PATH = pathlib.Path(os.environ.get("DEFTRI_LIB", PKG_ROOT / "libdeftri.so"))   # DEFTRI_LIB: dev builds
_lib = None


class DeftriError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"deftri error {code}: {msg}")
        self.code = code


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} not built — run __graft_entry__.build() (make -C csrc)")
    lib = C.CDLL(str(LIB_PATH))
    P = C.POINTER
    sig = {
        "deftri_abi_version": (C.c_int, []),
        "deftri_ctx_create": (C.c_int, [C.c_int32, P(C.c_void_p)]),
        "deftri_ctx_destroy": (C.c_int, [C.c_void_p]),
        "deftri_last_error": (C.c_char_p, [C.c_void_p]),
        "deftri_problem_upload": (C.c_int, [C.c_void_p, P(_abi.ProblemDesc)]),
        "deftri_problem_analyse": (C.c_int, [C.c_void_p, P(_abi.ProblemDesc)]),
        "deftri_plan_stats": (C.c_int, [C.c_void_p, P(_abi.Report)]),
        "deftri_debug_plan_solve": (C.c_int, [C.c_void_p, P(C.c_double), C.c_double, P(C.c_double),
                                              P(C.c_double), C.c_int64]),
        "deftri_solve_lm": (C.c_int, [C.c_void_p, P(_abi.LMParams), P(_abi.Report)]),
        "deftri_set_lm_lanes": (C.c_int, [C.c_void_p, C.c_int32]),
        "deftri_set_jacobian_mode": (C.c_int, [C.c_void_p, C.c_int32]),
        "deftri_set_factor_precision": (C.c_int, [C.c_void_p, C.c_int32]),
        "deftri_set_linear_solver": (C.c_int, [C.c_void_p, C.c_int32, C.c_double, C.c_int32]),
        "deftri_last_step_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
        "deftri_set_plan": (C.c_int, [C.c_void_p, C.c_int32]),
        "deftri_set_pair_window": (C.c_int, [C.c_void_p, C.c_int32]),
        "deftri_set_jacobian_storage": (C.c_int, [C.c_void_p, C.c_int32]),
        "deftri_get_plan_info": (C.c_int, [C.c_void_p, P(_abi.PlanInfo)]),
        "deftri_debug_sp_product": (C.c_int, [C.c_void_p, P(_abi.ProblemDesc), P(C.c_double), P(C.c_double),
                                              P(C.c_double), P(C.c_double), P(C.c_double), P(C.c_double),
                                              C.c_double, P(C.c_double), P(C.c_double), C.c_int64, P(C.c_int64)]),
        "deftri_pixels_stand_dev": (C.c_int, [C.c_void_p, P(_abi.MapC), P(_abi.PixelsError)]),
        "deftri_triangulate_nrslam": (C.c_int, [C.c_void_p, C.c_int32, P(C.c_float), P(C.c_float), P(C.c_float),
                                                P(C.c_float), P(C.c_float), P(C.c_float), C.c_float, P(C.c_float),
                                                P(C.c_float), P(C.c_uint8)]),
        "deftri_download": (C.c_int, [C.c_void_p, P(C.c_double), P(C.c_double), P(C.c_double)]),
        "deftri_reset_state": (C.c_int, [C.c_void_p]),
        "deftri_eval_chi2": (C.c_int, [C.c_void_p, P(C.c_double)]),
        "deftri_eval_gradient": (C.c_int, [C.c_void_p, P(C.c_double), P(C.c_double), C.c_int64]),
        "deftri_eval_hessian_product": (C.c_int, [C.c_void_p, P(C.c_double), P(C.c_double), C.c_int64]),
        "deftri_eval_damped_solve": (C.c_int, [C.c_void_p, C.c_double, P(C.c_double), P(C.c_double), C.c_int64]),
        "deftri_num_unknowns": (C.c_int64, [C.c_void_p]),
        "deftri_sizeof": (C.c_int64, [C.c_int32]),
        "deftri_profile_trial": (C.c_int, [C.c_void_p, C.c_double, P(_abi.KernelStat), C.c_int32, P(C.c_int32)]),
        "deftri_arap_graph_point_ids": (C.c_int, [C.c_void_p, P(C.c_int64), C.c_int64]),
        "deftri_graph_stats": (C.c_int, [C.c_void_p, P(C.c_int64), P(C.c_int64), P(C.c_double)]),
        "deftri_graph_repairs": (C.c_int, [C.c_void_p, P(C.c_int64), P(C.c_int64)]),
        "deftri_arap_build_graph": (C.c_int, [C.c_void_p, P(_abi.MapC), C.c_double, C.c_double, C.c_float,
                                              P(P(_abi.ProblemDesc))]),
        "deftri_arap_optimization": (C.c_int, [C.c_void_p, P(_abi.MapC), C.c_double, C.c_double, C.c_double,
                                               C.c_double, C.c_double, C.c_float, C.c_int32, P(C.c_double),
                                               P(_abi.Report)]),
        "deftri_deformation_optimization": (C.c_int, [C.c_void_p, P(_abi.MapC), P(_abi.DeformationParams),
                                                      P(_abi.DeformationReport)]),
        "deftri_global_insert": (C.c_int, [P(C.c_double), P(C.c_double), P(C.c_double)]),
        "deftri_keyframe_order": (C.c_int, [P(C.c_int64), C.c_int32, C.c_int32, P(C.c_int64)]),
        "deftri_debug_nelder_mead": (C.c_int, [_abi.OBJECTIVE_FN, C.c_void_p, C.c_int32, P(C.c_double), P(C.c_double),
                                               P(C.c_double), C.c_double, C.c_double, C.c_int32, P(C.c_double),
                                               P(C.c_int32), P(C.c_int32)]),
        # bundle adjustment
        "deftri_ba_create": (C.c_int, [C.c_int32, P(C.c_void_p)]),
        "deftri_ba_destroy": (C.c_int, [C.c_void_p]),
        "deftri_ba_last_error": (C.c_char_p, [C.c_void_p]),
        "deftri_ba_upload": (C.c_int, [C.c_void_p, P(_abi.BADesc)]),
        "deftri_ba_set_state": (C.c_int, [C.c_void_p, P(C.c_double), P(C.c_double)]),
        "deftri_ba_set_edge_flags": (C.c_int, [C.c_void_p, P(C.c_uint8), P(C.c_uint8)]),
        "deftri_ba_solve_lm": (C.c_int, [C.c_void_p, P(_abi.LMParams), C.c_int32, P(_abi.Report)]),
        "deftri_ba_compute_errors": (C.c_int, [C.c_void_p, P(C.c_uint8)]),
        "deftri_ba_edge_chi2": (C.c_int, [C.c_void_p, P(C.c_double), P(C.c_uint8)]),
        "deftri_ba_download": (C.c_int, [C.c_void_p, P(C.c_double), P(C.c_double)]),
        "deftri_ba_eval_system": (C.c_int, [C.c_void_p, C.c_int32, C.c_double, P(C.c_double), P(C.c_double),
                                            P(C.c_double), P(C.c_double), P(C.c_double), P(C.c_int32)]),
        "deftri_rccl_unique_id": (C.c_int, [P(C.c_uint8)]),
        "deftri_dist_init_rccl": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, P(C.c_uint8)]),
        "deftri_dist_set_transport": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, _abi.XFER_FN, C.c_void_p]),
        "deftri_dist_vertex_owner": (C.c_int, [C.c_void_p, P(C.c_int32), C.c_int64]),
        "deftri_plan_vertex_order": (C.c_int, [C.c_void_p, P(C.c_int64), C.c_int64]),
        "deftri_measure_sim_absolute_map_errors": (C.c_int, [C.c_int32, P(_abi.MapC), C.c_int32, P(C.c_float),
                                                             P(C.c_float), P(_abi.AbsErrorsC)]),
        "deftri_measure_relative_map_errors": (C.c_int, [C.c_int32, P(_abi.MapC), P(_abi.RelErrorsC), C.c_int32,
                                                         P(C.c_int32)]),
        "deftri_sim_normal_stream": (C.c_int, [C.c_int64, C.c_float, C.c_float, P(C.c_float)]),
        "deftri_sim_two_view": (C.c_int, [C.c_int32, P(C.c_float), P(C.c_float), P(C.c_float), P(C.c_float),
                                          P(C.c_float), P(C.c_float), C.c_float, C.c_int32, C.c_float, C.c_float,
                                          C.c_float, P(C.c_float), P(C.c_float), P(C.c_float), P(C.c_float),
                                          P(C.c_float), P(C.c_float)]),
        "deftri_dist_owned_edges": (C.c_int, [C.c_void_p, P(C.c_uint8), P(C.c_uint8), P(C.c_uint8)]),
        "deftri_debug_plan_solve_dist": (C.c_int, [C.c_void_p, P(C.c_double), C.c_double, P(C.c_double),
                                                   P(C.c_double), C.c_int64]),
        "deftri_ba_dist_init_rccl": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, P(C.c_uint8)]),
        "deftri_ba_dist_set_allreduce": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, _abi.ALLREDUCE_FN,
                                                   C.c_void_p]),
        "deftri_ba_profile_trial": (C.c_int, [C.c_void_p, C.c_double, P(_abi.KernelStat), C.c_int32,
                                              P(C.c_int32)]),
    }
    dev_build = "DEFTRI_LIB" in os.environ          # an older build under A/B may lack newer entry points
    for name, (res, args) in sig.items():
        if dev_build and not hasattr(lib, name):
            continue
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


EXPORTED = [
    "deftri_abi_version", "deftri_ctx_create", "deftri_ctx_destroy", "deftri_last_error",
    "deftri_problem_upload", "deftri_problem_analyse", "deftri_plan_stats", "deftri_debug_plan_solve",
    "deftri_solve_lm", "deftri_set_lm_lanes", "deftri_set_jacobian_mode", "deftri_set_factor_precision", "deftri_set_linear_solver", "deftri_last_step_info", "deftri_pixels_stand_dev", "deftri_triangulate_nrslam", "deftri_download", "deftri_reset_state", "deftri_eval_chi2",
    "deftri_eval_gradient", "deftri_eval_hessian_product", "deftri_eval_damped_solve",
    "deftri_num_unknowns", "deftri_sizeof", "deftri_arap_build_graph", "deftri_arap_graph_point_ids", "deftri_graph_stats", "deftri_graph_repairs", "deftri_arap_optimization",
    "deftri_profile_trial",
    "deftri_ba_create", "deftri_ba_destroy", "deftri_ba_last_error", "deftri_ba_upload", "deftri_ba_set_state",
    "deftri_ba_set_edge_flags", "deftri_ba_solve_lm", "deftri_ba_compute_errors", "deftri_ba_edge_chi2",
    "deftri_ba_download", "deftri_ba_eval_system", "deftri_rccl_unique_id", "deftri_ba_dist_init_rccl",
    "deftri_ba_dist_set_allreduce", "deftri_ba_profile_trial",
    "deftri_dist_init_rccl", "deftri_dist_set_transport", "deftri_dist_vertex_owner", "deftri_plan_vertex_order", "deftri_sim_two_view", "deftri_sim_normal_stream",
    "deftri_measure_sim_absolute_map_errors", "deftri_measure_relative_map_errors", "deftri_dist_owned_edges",
    "deftri_debug_plan_solve_dist", "deftri_set_plan", "deftri_set_jacobian_storage", "deftri_get_plan_info",
    "deftri_debug_sp_product", "deftri_set_pair_window", "deftri_deformation_optimization", "deftri_global_insert",
    "deftri_debug_nelder_mead", "deftri_keyframe_order",
]


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Context:
    """One solver context (one per host thread).  device < 0 = host-only (graph / analysis)."""

    def __init__(self, device=0):
        self.h = None                    # close() / __del__ after a failed create
        self.lib = load()
        h = C.c_void_p()
        rc = self.lib.deftri_ctx_create(int(device), C.byref(h))
        if rc != 0:
            raise DeftriError(rc, "deftri_ctx_create failed (no usable gfx950 device?)" if device >= 0 else "ctx")
        self.h = h
        self.device = device
        self._desc = None
        self._prob = None
        self._solver = ("pcg", 0.0, 0)
        self.jacobian_mode = False       # deftri_set_jacobian_mode's default: g2o numeric Jacobians

    def set_jacobian_mode(self, analytic):
        """The Jacobians of deftri_arap_optimization / _deformation_optimization on this context."""
        self._check(self.lib.deftri_set_jacobian_mode(self.h, 1 if analytic else 0))
        self.jacobian_mode = bool(analytic)

    def close(self):
        if getattr(self, "h", None):
            self.lib.deftri_ctx_destroy(self.h)
            self.h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc):
        if rc != 0:
            raise DeftriError(rc, (self.lib.deftri_last_error(self.h) or b"").decode())

    # flat-graph API ------------------------------------------------------------------------
    def upload(self, prob: Problem):
        self._prob = prob
        self._desc = prob.to_desc()
        self._check(self.lib.deftri_problem_upload(self.h, C.byref(self._desc)))

    def analyse(self, prob: Problem):
        self._prob = prob
        self._desc = prob.to_desc()
        self._check(self.lib.deftri_problem_analyse(self.h, C.byref(self._desc)))

    def plan_stats(self):
        r = _abi.Report()
        self._check(self.lib.deftri_plan_stats(self.h, C.byref(r)))
        return {k: v for k, v in r.as_dict().items() if k in ("n_unknowns", "nnz_factor", "factor_flops", "n_fronts", "n_levels")}

    def debug_plan_solve(self, H, lam, rhs):
        H = np.ascontiguousarray(H, dtype=np.float64)
        r = np.ascontiguousarray(rhs, dtype=np.float64)
        x = np.zeros_like(r)
        self._check(self.lib.deftri_debug_plan_solve(self.h, _dp(H), float(lam), _dp(r), _dp(x), len(r)))
        return x

    # point-sharded solve ---------------------------------------------------------------------
    def dist_init_rccl(self, nranks, rank, uid):
        """RCCL communicator (uid: 128 bytes from rccl_unique_id() on rank 0)."""
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(uid))
        self._check(self.lib.deftri_dist_init_rccl(self.h, int(nranks), int(rank), buf))

    def dist_set_transport(self, nranks, rank, transport):
        """Host-memory transport: `transport(op, peer, array)` with op 0 sum / 1 max all-reduce in
        place, 2 send, 3 receive (array: float64 view of the staging buffer); returns 0."""
        def cb(_user, op, peer, buf, n):
            try:
                arr = np.ctypeslib.as_array(buf, shape=(int(n),)) if n > 0 else np.zeros(0)
                return int(transport(int(op), int(peer), arr) or 0)
            except Exception as e:           # never let an exception cross the C frames
                import sys
                print(f"deftri transport callback failed: {e!r}", file=sys.stderr, flush=True)
                return -1
        self._xfer_cb = _abi.XFER_FN(cb) if nranks > 1 else _abi.XFER_FN()
        self._check(self.lib.deftri_dist_set_transport(self.h, int(nranks), int(rank), self._xfer_cb, None))

    def vertex_owner(self):
        nv = self._prob.n_pairs + self._prob.n_scales + self._prob.n_points
        out = np.zeros(nv, np.int32)
        self._check(self.lib.deftri_dist_vertex_owner(self.h, out.ctypes.data_as(C.POINTER(C.c_int32)), nv))
        return out

    def vertex_order(self):
        nv = self._prob.n_pairs + self._prob.n_scales + self._prob.n_points
        out = np.zeros(nv, np.int64)
        self._check(self.lib.deftri_plan_vertex_order(self.h, out.ctypes.data_as(C.POINTER(C.c_int64)), nv))
        return out

    def owned_edges(self):
        p = self._prob
        r, d, a = (np.zeros(max(k, 1), np.uint8) for k in (len(p.rep_point), len(p.dep_point), len(p.arap_pair)))
        u8 = lambda x: x.ctypes.data_as(C.POINTER(C.c_uint8))
        self._check(self.lib.deftri_dist_owned_edges(self.h, u8(r), u8(d), u8(a)))
        return (r[:len(p.rep_point)].astype(bool), d[:len(p.dep_point)].astype(bool), a[:len(p.arap_pair)].astype(bool))

    def debug_plan_solve_dist(self, Hq, lam, bq):
        Hq = np.ascontiguousarray(Hq, dtype=np.float64)
        bq = np.ascontiguousarray(bq, dtype=np.float64)
        x = np.zeros_like(bq)
        self._check(self.lib.deftri_debug_plan_solve_dist(self.h, _dp(Hq), float(lam), _dp(bq), _dp(x), len(bq)))
        return x

    def set_linear_solver(self, solver="pcg", tol=0.0, max_iterations=0):
        """LM step solver: "pcg" (block-Jacobi PCG, LDL^T fallback; default) or "direct" (multifrontal LDL^T)."""
        code = {"direct": _abi.DEFTRI_SOLVER_DIRECT, "pcg": _abi.DEFTRI_SOLVER_PCG}[solver]
        self._check(self.lib.deftri_set_linear_solver(self.h, code, float(tol), int(max_iterations)))
        self._solver = (solver, tol, max_iterations)

    def set_plan(self, plan="auto"):
        """Plan kind of the next upload: "auto", "multifrontal" (LDL^T analysis; sliced matrix-free PCG
        where it fits) or "iterative" (point-sharded matrix-free PCG, no factorization; csrc/spcg.h)."""
        code = {"auto": _abi.DEFTRI_PLAN_AUTO, "multifrontal": _abi.DEFTRI_PLAN_MULTIFRONTAL,
                "iterative": _abi.DEFTRI_PLAN_ITERATIVE}[plan]
        self._check(self.lib.deftri_set_plan(self.h, code))

    def set_pair_window(self, window):
        """Graph builds: 0 every keyframe pair (the reference), w > 0 pairs at most w apart in map order."""
        self._check(self.lib.deftri_set_pair_window(self.h, int(window)))

    def set_jacobian_storage(self, fp32):
        """Iterative plan: the ARAP Jacobians the product reads in fp32 (1) or fp64 (0, default)."""
        self._check(self.lib.deftri_set_jacobian_storage(self.h, 1 if fp32 else 0))

    def plan_info(self):
        info = _abi.PlanInfo()
        self._check(self.lib.deftri_get_plan_info(self.h, C.byref(info)))
        return info.as_dict()

    def debug_sp_product(self, prob, jarap, warap, jrep, wrep, jdep, wdep, lam, p):
        """Host emulation of the iterative plan's product on this rank (deftri_debug_sp_product):
        returns (q with this rank's rows + the global vertices, [own rows, halo rows, local ARAP
        edges, owned ARAP edges])."""
        d = prob.to_desc()
        f = lambda a: np.ascontiguousarray(a, dtype=np.float64)
        arrs = [f(a) for a in (jarap, warap, jrep, wrep, jdep, wdep, p)]
        q = np.zeros(prob.n_unknowns)
        st = np.zeros(4, np.int64)
        self._check(self.lib.deftri_debug_sp_product(self.h, C.byref(d), *[_dp(a) for a in arrs[:6]], float(lam),
                                                     _dp(arrs[6]), _dp(q), prob.n_unknowns,
                                                     st.ctypes.data_as(C.POINTER(C.c_int64))))
        return q, st

    def last_step_info(self):
        """(CG iterations, converged) of the last PCG step."""
        it, ok = C.c_int32(), C.c_int32()
        self._check(self.lib.deftri_last_step_info(self.h, C.byref(it), C.byref(ok)))
        return it.value, bool(ok.value)

    def set_factor_precision(self, fp32_updates):
        """1: trailing updates on fp32 MFMA (the C5 precision sweep); 0: fp64 (default, the reference's)."""
        self._check(self.lib.deftri_set_factor_precision(self.h, 1 if fp32_updates else 0))

    def set_lm_lanes(self, lanes):
        """Speculative lambda lanes (0 = default, 1 = sequential trials); results are identical."""
        self._check(self.lib.deftri_set_lm_lanes(self.h, int(lanes)))

    def solve_lm(self, n_iterations=10, analytic=False, tau=1e-5, max_trials=10, user_lambda=0.0, verbose=False):
        prm = _abi.LMParams(n_iterations=n_iterations, max_trials=max_trials, tau=tau, user_lambda=user_lambda,
                            analytic_jacobians=1 if analytic else 0, verbose=1 if verbose else 0)
        rep = _abi.Report()
        self._check(self.lib.deftri_solve_lm(self.h, C.byref(prm), C.byref(rep)))
        return rep.as_dict()

    def download(self):
        p = self._prob
        pts = np.zeros((p.n_points, 3)); sc = np.zeros(p.n_scales); tg = np.zeros((p.n_pairs, 7))
        self._check(self.lib.deftri_download(self.h, _dp(pts), _dp(sc), _dp(tg)))
        return pts, sc, tg

    def reset_state(self):
        self._check(self.lib.deftri_reset_state(self.h))

    def chi2(self):
        v = C.c_double()
        self._check(self.lib.deftri_eval_chi2(self.h, C.byref(v)))
        return v.value

    def gradient(self):
        n = self._prob.n_unknowns
        b = np.zeros(n); d = np.zeros(n)
        self._check(self.lib.deftri_eval_gradient(self.h, _dp(b), _dp(d), n))
        return b, d

    def hessian_product(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros_like(x)
        self._check(self.lib.deftri_eval_hessian_product(self.h, _dp(x), _dp(y), len(x)))
        return y

    def damped_solve(self, lam, rhs, solver="direct", tol=0.0, max_iterations=0):
        """(H + lam I) x = rhs with `solver` ("direct" LDL^T or "pcg"); the context's solver setting
        is restored afterwards."""
        r = np.ascontiguousarray(rhs, dtype=np.float64)
        x = np.zeros_like(r)
        prev = self._solver
        self.set_linear_solver(solver, tol, max_iterations)
        try:
            self._check(self.lib.deftri_eval_damped_solve(self.h, float(lam), _dp(r), _dp(x), len(r)))
        finally:
            self.set_linear_solver(*prev)
        return x

    def profile_trial(self, lam):
        """Per-kernel device time of one LM trial: {name: {launches, ms, flops, bytes}}."""
        arr = (_abi.KernelStat * 64)()
        n = C.c_int32()
        self._check(self.lib.deftri_profile_trial(self.h, float(lam), arr, 64, C.byref(n)))
        return {arr[i].name.decode(): {"launches": arr[i].launches, "ms": arr[i].ms, "flops": arr[i].flops,
                                       "bytes": arr[i].bytes} for i in range(n.value)}

    # map-level API -------------------------------------------------------------------------
    def build_graph(self, m, rep_weight, arap_weight, depth_error):
        mc, keep = m.to_c()
        out = C.POINTER(_abi.ProblemDesc)()
        self._check(self.lib.deftri_arap_build_graph(self.h, C.byref(mc), float(rep_weight), float(arap_weight),
                                                     C.c_float(depth_error), C.byref(out)))
        p = Problem.from_desc(out.contents)
        ids = np.zeros(p.n_points, np.int64)
        self._check(self.lib.deftri_arap_graph_point_ids(self.h, ids.ctypes.data_as(C.POINTER(C.c_int64)), p.n_points))
        p.point_ids = ids
        return p

    def graph_repairs(self):
        """(keyframe meshes of full graph builds repaired from the previous build's triangulation, their
        flips) over this context's life."""
        a, b = C.c_int64(), C.c_int64()
        self._check(self.lib.deftri_graph_repairs(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def graph_stats(self):
        """(memo hits, structure-memo hits, host ms of the last graph build)."""
        a, b, t = C.c_int64(), C.c_int64(), C.c_double()
        self._check(self.lib.deftri_graph_stats(self.h, C.byref(a), C.byref(b), C.byref(t)))
        return a.value, b.value, t.value

    def pixels_stand_dev(self, m):
        """calculatePixelsStandDev (Geometry.cc:370-498) of a Map on the device."""
        mc, keep = m.to_c()
        out = _abi.PixelsError()
        self._check(self.lib.deftri_pixels_stand_dev(self.h, C.byref(mc), C.byref(out)))
        return out.as_dict()

    def triangulate_nrslam(self, uv1, uv2, kb8_1, kb8_2, T1w, T2w, min_cos=0.9998):
        """Mapping::triangulateSimulatedMapPoints (NRSLAM, FarPoints) on the device.  T1w/T2w: SE3f
        (R, t).  Returns (x3d_1 [n,3], x3d_2 [n,3], valid [n] bool), fp32."""
        f = lambda a: np.ascontiguousarray(a, np.float32)
        uv1, uv2 = f(uv1), f(uv2)
        n = len(uv1)
        T = [f(np.concatenate([np.asarray(Tx.R, np.float32), np.asarray(Tx.t, np.float32)[:, None]], 1)) for Tx in (T1w, T2w)]
        k1, k2 = f(kb8_1), f(kb8_2)
        x1 = np.zeros((n, 3), np.float32); x2 = np.zeros((n, 3), np.float32); v = np.zeros(n, np.uint8)
        fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))
        self._check(self.lib.deftri_triangulate_nrslam(self.h, n, fp(uv1), fp(uv2), fp(k1), fp(k2), fp(T[0]), fp(T[1]),
                                                      float(min_cos), fp(x1), fp(x2),
                                                      v.ctypes.data_as(C.POINTER(C.c_uint8))))
        return x1, x2, v.astype(bool)

    def arap_optimization(self, m, rep_weight, global_weight, arap_weight, alpha, beta, depth_error,
                          n_iterations, want_update=True, analytic=False):
        """analytic=False (default): g2o numeric ARAP/depth Jacobians, the reference's arithmetic."""
        prev = self.jacobian_mode
        self.set_jacobian_mode(analytic)
        mc, keep = m.to_c()
        upd = C.c_double(0.0)
        rep = _abi.Report()
        t = time.perf_counter()
        try:
            rc = self.lib.deftri_arap_optimization(
                self.h, C.byref(mc), float(rep_weight), float(global_weight), float(arap_weight), float(alpha),
                float(beta), C.c_float(depth_error), int(n_iterations), C.byref(upd) if want_update else None,
                C.byref(rep))
        finally:
            self.set_jacobian_mode(prev)               # the caller's mode again
        self.last_call_s = time.perf_counter() - t     # the C-ABI call alone (no Python marshalling)
        self._check(rc)
        m.from_c(mc, keep)
        return upd.value, rep.as_dict()


    def deformation_optimization(self, m, settings, max_evals=4096):
        """deformationOptimization (g2oBundleAdjustment.cc:446-606) in native code
        (deftri_deformation_optimization): the outer rounds, the Nelder-Mead weight search on map
        clones, arapOptimization and calculatePixelsStandDev on the device.  Writes the map back
        (positions, depth scales, the global table) and returns the report as a dict with the
        evaluation log."""
        settings.validate_for_solver()
        if settings.selection == "open3DArap":
            raise NotImplementedError("open3DArap (Open3D DeformAsRigidAsPossible) is out of scope")
        prm = _abi.DeformationParams()
        # any other selection is the fixed-weight round (:565-568); "twoOptimizations" with a
        # weightsSelection other than "nlopt" too (the Eigen LM returns before evaluating, deftri.h)
        prm.selection = 1 if (settings.selection == "twoOptimizations" and settings.weights_selection == "nlopt") else 0
        prm.rep, prm.global_, prm.arap = float(settings.rep), float(settings.global_), float(settings.arap)
        prm.alpha, prm.beta = float(settings.alpha), float(settings.beta)
        prm.depth_error = float(settings.depth_sigma)
        prm.n_iterations, prm.n_optimizations = int(settings.n_iterations), int(settings.n_optimizations)
        prm.lb[:] = [settings.nlopt_rep_lb, settings.nlopt_global_lb, settings.nlopt_arap_lb]
        prm.ub[:] = [settings.nlopt_rep_ub, settings.nlopt_global_ub, settings.nlopt_arap_ub]
        prm.xtol_rel, prm.xtol_abs = float(settings.nlopt_rel_tol), float(settings.nlopt_abs_tol)
        prm.maxeval = int(settings.nlopt_iterations)
        prm.n_map_points = len(m.map_points)
        evals = (_abi.DeformationEval * max_evals)()
        rep = _abi.DeformationReport()
        rep.evals = C.cast(evals, C.POINTER(_abi.DeformationEval))
        rep.max_evals = max_evals
        mc, keep = m.to_c()
        prev = self.jacobian_mode
        self.set_jacobian_mode(False)                  # g2o numeric J (the reference's)
        t = time.perf_counter()
        try:
            rc = self.lib.deftri_deformation_optimization(self.h, C.byref(mc), C.byref(prm), C.byref(rep))
        finally:
            self.set_jacobian_mode(prev)               # the caller's mode again
        self.last_call_s = time.perf_counter() - t
        self._check(rc)
        if rep.rounds > 0:
            m.from_c(mc, keep)
        ev = [{"round": evals[k].round, "eval": evals[k].eval, "x": list(evals[k].x), "f": evals[k].f}
              for k in range(min(rep.n_evals, max_evals))]
        return {"rounds": rep.rounds, "arap_calls": rep.arap_calls, "weights": list(rep.weights), "minf": rep.minf,
                "nlopt_result": rep.nlopt_result, "update": rep.update, "seconds": rep.seconds, "evaluations": ev,
                "round_update": list(rep.round_update[:min(rep.rounds, 64)]),
                "round_weights": [list(rep.round_weights[k]) for k in range(min(rep.rounds, 64))]}


def keyframe_order(insert_ids, clones=0):
    """deftri_keyframe_order: the iteration order of Map::mKeyFrames_ (std::unordered_map<ID,
    KeyFrame_>) after inserting `insert_ids` in order, then `clones` Map::clone re-insertions."""
    lib = load()
    n = len(insert_ids)
    a = (C.c_int64 * max(n, 1))(*[int(v) for v in insert_ids])
    out = (C.c_int64 * max(n, 1))()
    rc = lib.deftri_keyframe_order(a, n, int(clones), out)
    if rc:
        raise DeftriError(rc, "deftri_keyframe_order")
    return [int(out[k]) for k in range(n)]


def global_insert(t7):
    """deftri_global_insert: the (0, 1) and (1, 0) entries Map::insertGlobalKeyFramesTransformation
    stores for the solved T_g, as the 7-vectors the next arapOptimization reads (host, no GPU)."""
    lib = load()
    a = (C.c_double * 7)(*[float(v) for v in t7])
    f, i = (C.c_double * 7)(), (C.c_double * 7)()
    rc = lib.deftri_global_insert(a, f, i)
    if rc:
        raise DeftriError(rc, "deftri_global_insert")
    return list(f), list(i)


def nelder_mead_native(f, x0, lb, ub, xtol_rel=0.0, xtol_abs=0.0, maxeval=0):
    """deftri_debug_nelder_mead: the native restated NLopt LN_NELDERMEAD on a Python objective (tests)."""
    lib = load()
    n = len(x0)
    x = (C.c_double * n)(*map(float, x0))
    lo, hi = (C.c_double * n)(*map(float, lb)), (C.c_double * n)(*map(float, ub))
    seen = []

    def cb(xp, nn, user):
        xv = [xp[k] for k in range(nn)]
        seen.append(xv)
        return float(f(xv))
    fn = _abi.OBJECTIVE_FN(cb)
    minf, nev, res = C.c_double(), C.c_int32(), C.c_int32()
    rc = lib.deftri_debug_nelder_mead(fn, None, n, x, lo, hi, float(xtol_rel), float(xtol_abs), int(maxeval),
                                      C.byref(minf), C.byref(nev), C.byref(res))
    if rc:
        raise DeftriError(rc, "deftri_debug_nelder_mead")
    return list(x), minf.value, res.value, nev.value, seen


class BAContext:
    """Bundle-adjustment solver context on one GPU (deftri_ba_*).  `prob` is a ba.BAProblem."""

    def __init__(self, device=0):
        self.h = None                    # close() / __del__ after a failed create
        self.lib = load()
        h = C.c_void_p()
        rc = self.lib.deftri_ba_create(int(device), C.byref(h))
        if rc != 0:
            raise DeftriError(rc, "deftri_ba_create failed (no usable gfx950 device?)")
        self.h = h
        self.device = device
        self._prob = None
        self._desc = None
        self._cb = None

    def close(self):
        if getattr(self, "h", None):
            self.lib.deftri_ba_destroy(self.h)
            self.h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc):
        if rc != 0:
            raise DeftriError(rc, (self.lib.deftri_ba_last_error(self.h) or b"").decode())

    def upload(self, prob):
        self._prob = prob
        self._desc = prob.to_desc()
        self._check(self.lib.deftri_ba_upload(self.h, C.byref(self._desc)))

    def set_state(self, poses=None, points=None):
        p = None if poses is None else np.ascontiguousarray(poses, np.float64)
        q = None if points is None else np.ascontiguousarray(points, np.float64)
        self._check(self.lib.deftri_ba_set_state(self.h, None if p is None else _dp(p), None if q is None else _dp(q)))

    def set_edge_flags(self, level=None, robust=None):
        lv = None if level is None else np.ascontiguousarray(level, np.uint8)
        rb = None if robust is None else np.ascontiguousarray(robust, np.uint8)
        self._check(self.lib.deftri_ba_set_edge_flags(self.h, _abi.ptr(lv, C.c_uint8), _abi.ptr(rb, C.c_uint8)))

    def solve_lm(self, n_iterations=10, level=0, tau=1e-5, max_trials=10, user_lambda=0.0, verbose=False):
        prm = _abi.LMParams(n_iterations=n_iterations, max_trials=max_trials, tau=tau, user_lambda=user_lambda,
                            analytic_jacobians=1, verbose=1 if verbose else 0)
        rep = _abi.Report()
        self._check(self.lib.deftri_ba_solve_lm(self.h, C.byref(prm), int(level), C.byref(rep)))
        return rep.as_dict()

    def compute_errors(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        self._check(self.lib.deftri_ba_compute_errors(self.h, _abi.ptr(m, C.c_uint8)))

    def edge_chi2(self):
        n = self._prob.n_edges
        chi = np.zeros(n); dp = np.zeros(n, np.uint8)
        self._check(self.lib.deftri_ba_edge_chi2(self.h, _dp(chi), _abi.ptr(dp, C.c_uint8)))
        return chi, dp.astype(bool)

    def download(self):
        p = self._prob
        poses = np.zeros((p.n_poses, 7)); pts = np.zeros((p.n_points, 3))
        self._check(self.lib.deftri_ba_download(self.h, _dp(poses), _dp(pts)))
        return poses, pts

    def eval_system(self, lam, level=0):
        p = self._prob
        K, P = p.n_poses, p.n_points
        ns_max = 6 * K
        S = np.zeros((ns_max, ns_max)); rhs = np.zeros(ns_max)
        dx = np.zeros(6 * K + 3 * P); b = np.zeros(6 * K + 3 * P)
        chi = C.c_double(); ns = C.c_int32()
        self._check(self.lib.deftri_ba_eval_system(self.h, int(level), float(lam), C.byref(chi), _dp(S), _dp(rhs),
                                                   _dp(dx), _dp(b), C.byref(ns)))
        n = ns.value
        S = S.reshape(-1)[:n * n].reshape(n, n).copy()
        return {"chi2": chi.value, "S": S, "rhs": rhs[:n].copy(), "dx": dx, "b": b, "ns": n}

    def dist_init_rccl(self, nranks, rank, uid):
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(uid))
        self._check(self.lib.deftri_ba_dist_init_rccl(self.h, int(nranks), int(rank), buf))

    def dist_set_allreduce(self, nranks, rank, fn):
        """fn(np.ndarray view of the host buffer, op) -> None, reducing in place (op 0 sum, 1 max)."""
        def _cb(user, buf, n, op):
            try:
                fn(np.ctypeslib.as_array(buf, shape=(n,)), int(op))
                return 0
            except Exception:                       # noqa: BLE001 — reported as a failed call
                import traceback
                traceback.print_exc()
                return 1
        self._cb = _abi.ALLREDUCE_FN(_cb)
        self._check(self.lib.deftri_ba_dist_set_allreduce(self.h, int(nranks), int(rank), self._cb, None))

    def profile_trial(self, lam):
        arr = (_abi.KernelStat * 64)()
        n = C.c_int32()
        self._check(self.lib.deftri_ba_profile_trial(self.h, float(lam), arr, 64, C.byref(n)))
        return {arr[i].name.decode(): {"launches": arr[i].launches, "ms": arr[i].ms, "flops": arr[i].flops,
                                       "bytes": arr[i].bytes} for i in range(n.value)}


def sim_two_view(orig, moved, c1, c2, kb8_1, kb8_2, rep_error, decimals, depth_error_mm, depth_scales):
    """deftri_sim_two_view: the reference's simulated keypoints / depths / camera poses (SLAM.cc:223-338)."""
    lib = load()
    f32 = lambda a: np.ascontiguousarray(a, np.float32)
    orig, moved = f32(orig).reshape(-1, 3), f32(moved).reshape(-1, 3)
    n = len(orig)
    c1, c2, k1, k2 = f32(c1), f32(c2), f32(kb8_1), f32(kb8_2)
    uv1 = np.zeros((n, 2), np.float32); uv2 = np.zeros((n, 2), np.float32)
    d1 = np.zeros(n, np.float32); d2 = np.zeros(n, np.float32)
    p1 = np.zeros(7, np.float32); p2 = np.zeros(7, np.float32)
    fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))
    rc = lib.deftri_sim_two_view(n, fp(orig), fp(moved), fp(c1), fp(c2), fp(k1), fp(k2), float(rep_error),
                                 int(decimals), float(depth_error_mm), float(depth_scales[0]),
                                 float(depth_scales[1]), fp(uv1), fp(uv2), fp(d1), fp(d2), fp(p1), fp(p2))
    if rc != 0:
        raise DeftriError(rc, "deftri_sim_two_view")
    return uv1, uv2, d1, d2, p1, p2


def measure_sim_absolute(m, original, moved, device=0):
    """deftri_measure_sim_absolute_map_errors (Measurements.cc:8-98); values in mm."""
    lib = load()
    mc, keep = m.to_c()
    o = np.ascontiguousarray(original, np.float32).reshape(-1, 3)
    mv = np.ascontiguousarray(moved, np.float32).reshape(-1, 3)
    out = _abi.AbsErrorsC()
    fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))
    rc = lib.deftri_measure_sim_absolute_map_errors(int(device), C.byref(mc), len(o), fp(o), fp(mv), C.byref(out))
    if rc != 0:
        raise DeftriError(rc, "deftri_measure_sim_absolute_map_errors")
    return {k: getattr(out, k) for k, _ in _abi.AbsErrorsC._fields_}


def measure_relative(m, device=0):
    """deftri_measure_relative_map_errors (Measurements.cc:350-518): one record per keyframe pair."""
    lib = load()
    mc, keep = m.to_c()
    K = len(m.keyframes)
    npair = max(1, K * (K - 1) // 2)
    out = (_abi.RelErrorsC * npair)()
    n = C.c_int32()
    rc = lib.deftri_measure_relative_map_errors(int(device), C.byref(mc), out, npair, C.byref(n))
    if rc != 0:
        raise DeftriError(rc, "deftri_measure_relative_map_errors")
    return [{k: getattr(out[i], k) for k, _ in _abi.RelErrorsC._fields_} for i in range(n.value)]


def rccl_unique_id():
    lib = load()
    buf = (C.c_uint8 * 128)()
    rc = lib.deftri_rccl_unique_id(buf)
    if rc != 0:
        raise DeftriError(rc, "ncclGetUniqueId failed")
    return bytes(buf)
