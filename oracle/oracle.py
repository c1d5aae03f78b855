"""oracle.py — TEST INFRASTRUCTURE ONLY: ctypes binding of oracle/liboracle.so (the CPU
restatement of the reference LM path, deftri_oracle.c).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg."""
import ctypes as C
import os
import pathlib
import subprocess

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        so = HERE / "liboracle.so"
        if not so.exists():
            build()
        _lib = C.CDLL(str(so))
    return _lib


def _abi():
    from deftri import _abi as A
    return A


def _p(a, t):
    return None if a is None else a.ctypes.data_as(C.POINTER(t))


def chi2(prob, points=None, scales=None, tg=None):
    d = prob.to_desc()
    out = C.c_double()
    lib().oracle_chi2(C.byref(d), _p(points, C.c_double), _p(scales, C.c_double), _p(tg, C.c_double),
                      C.byref(out))
    return out.value


def edge_errors(prob):
    d = prob.to_desc()
    rep = np.zeros((len(prob.rep_point), 2)); dep = np.zeros(len(prob.dep_point))
    arap = np.zeros(len(prob.arap_pair))
    lib().oracle_edge_errors(C.byref(d), _p(rep, C.c_double), _p(dep, C.c_double), _p(arap, C.c_double))
    return rep, dep, arap


def arap_jacobians(prob, analytic=True):
    d = prob.to_desc()
    J = np.zeros((len(prob.arap_pair), 18))
    lib().oracle_arap_jacobians(C.byref(d), C.c_int(1 if analytic else 0), _p(J, C.c_double))
    return J


def linearize(prob, analytic=True, dense=False, x=None):
    d = prob.to_desc()
    n = prob.n_unknowns
    b = np.zeros(n)
    H = np.zeros((n, n)) if dense else None
    y = np.zeros(n) if x is not None else None
    xx = None if x is None else np.ascontiguousarray(x, dtype=np.float64)
    lib().oracle_linearize(C.byref(d), C.c_int(1 if analytic else 0), _p(b, C.c_double),
                           _p(H, C.c_double), _p(xx, C.c_double), _p(y, C.c_double))
    return b, H, y


def hessian_coo(prob, analytic=True):
    """(rows, cols, vals) of H at the initial linearization, every stored block entry."""
    d = prob.to_desc()
    n = C.c_int64(0)
    lib().oracle_hessian_coo(C.byref(d), C.c_int(1 if analytic else 0), C.byref(n), None, None, None)
    ri = np.zeros(n.value, np.int64); ci = np.zeros(n.value, np.int64); v = np.zeros(n.value)
    lib().oracle_hessian_coo(C.byref(d), C.c_int(1 if analytic else 0), C.byref(n), _p(ri, C.c_int64),
                             _p(ci, C.c_int64), _p(v, C.c_double))
    return ri, ci, v


def damped_solve(prob, lam, rhs, analytic=True):
    d = prob.to_desc()
    x = np.zeros(prob.n_unknowns)
    r = np.ascontiguousarray(rhs, dtype=np.float64)
    rc = lib().oracle_damped_solve(C.byref(d), C.c_int(1 if analytic else 0), C.c_double(lam),
                                   _p(r, C.c_double), _p(x, C.c_double))
    if rc != 0:
        raise ArithmeticError("oracle LDL^T: zero pivot")
    return x


def set_vertex_order(order):
    """Elimination order (vertex eliminated k-th) for the oracle's LDL^T; None restores its own
    nested dissection."""
    if order is None:
        lib().oracle_set_vertex_order(None, C.c_int64(0))
        return
    o = np.ascontiguousarray(order, dtype=np.int64)
    lib().oracle_set_vertex_order(_p(o, C.c_int64), C.c_int64(len(o)))


def set_edge_order(reversed_):
    """The order of the chi2 sums and of the H / b accumulation: the descriptor's (False, g2o's
    insertion order) or every edge type walked backwards (True; tools/oracle_spread.py)."""
    lib().oracle_set_edge_order(C.c_int(1 if reversed_ else 0))


def solve_lm(prob, n_iterations=10, analytic=False, tau=1e-5, max_trials=10, verbose=False):
    A = _abi()
    d = prob.to_desc()
    prm = A.LMParams(n_iterations=n_iterations, max_trials=max_trials, tau=tau, user_lambda=0.0,
                     analytic_jacobians=1 if analytic else 0, verbose=1 if verbose else 0)
    rep = A.Report()
    pts = np.zeros((prob.n_points, 3)); sc = np.zeros(prob.n_scales); tg = np.zeros((prob.n_pairs, 7))
    lib().oracle_solve_lm(C.byref(d), C.byref(prm), _p(pts, C.c_double), _p(sc, C.c_double),
                          _p(tg, C.c_double), C.byref(rep))
    return {"points": pts, "scales": sc, "tg": tg, "report": rep.as_dict()}


# ---- bundle adjustment (ba_oracle.c) ------------------------------------------------------
def _u8(a):
    return None if a is None else np.ascontiguousarray(a, np.uint8).ctypes.data_as(C.POINTER(C.c_uint8))


def ba_solve(prob, n_iterations=10, level=0, edge_level=None, edge_robust=None, poses=None, points=None, err=None,
             tau=1e-5, max_trials=10, verbose=False):
    """initializeOptimization(level); optimize(n) on a BAProblem; state and cached errors in/out."""
    A = _abi()
    d = prob.to_desc()
    prm = A.LMParams(n_iterations=n_iterations, max_trials=max_trials, tau=tau, user_lambda=0.0,
                     analytic_jacobians=1, verbose=1 if verbose else 0)
    rep = A.Report()
    ps = np.array(prob.poses if poses is None else poses, np.float64, copy=True)
    pt = np.array(prob.points if points is None else points, np.float64, copy=True)
    er = np.zeros((prob.n_edges, 2)) if err is None else np.array(err, np.float64, copy=True)
    lv = prob.edge_level if edge_level is None else edge_level
    rb = prob.edge_robust if edge_robust is None else edge_robust
    lib().oracle_ba_solve(C.byref(d), _u8(lv), _u8(rb), C.c_int32(level), C.byref(prm), _p(ps, C.c_double),
                          _p(pt, C.c_double), _p(er, C.c_double), C.byref(rep))
    return {"poses": ps, "points": pt, "err": er, "report": rep.as_dict()}


def ba_compute_errors(prob, poses, points):
    d = prob.to_desc()
    er = np.zeros((prob.n_edges, 2))
    ps = np.ascontiguousarray(poses, np.float64); pt = np.ascontiguousarray(points, np.float64)
    lib().oracle_ba_compute_errors(C.byref(d), _p(ps, C.c_double), _p(pt, C.c_double), _p(er, C.c_double))
    return er


def ba_edge_chi2(prob, poses, points, err):
    d = prob.to_desc()
    chi = np.zeros(prob.n_edges); dp = np.zeros(prob.n_edges, np.uint8)
    ps = np.ascontiguousarray(poses, np.float64); pt = np.ascontiguousarray(points, np.float64)
    er = np.ascontiguousarray(err, np.float64)
    lib().oracle_ba_edge_chi2(C.byref(d), _p(ps, C.c_double), _p(pt, C.c_double), _p(er, C.c_double),
                              _p(chi, C.c_double), dp.ctypes.data_as(C.POINTER(C.c_uint8)))
    return chi, dp.astype(bool)


def ba_eval_system(prob, lam, level=0, edge_level=None, edge_robust=None):
    d = prob.to_desc()
    K, P = prob.n_poses, prob.n_points
    S = np.zeros((6 * K, 6 * K)); rhs = np.zeros(6 * K); dx = np.zeros(6 * K + 3 * P); b = np.zeros(6 * K + 3 * P)
    chi = C.c_double(); ns = C.c_int32()
    lv = prob.edge_level if edge_level is None else edge_level
    rb = prob.edge_robust if edge_robust is None else edge_robust
    rc = lib().oracle_ba_eval_system(C.byref(d), _u8(lv), _u8(rb), C.c_int32(level), _p(prob.poses, C.c_double),
                                     _p(prob.points, C.c_double), C.c_double(lam), C.byref(chi), _p(S, C.c_double),
                                     _p(rhs, C.c_double), _p(dx, C.c_double), _p(b, C.c_double), C.byref(ns))
    n = ns.value
    return {"chi2": chi.value, "S": S.reshape(-1)[:n * n].reshape(n, n).copy(), "rhs": rhs[:n].copy(), "dx": dx,
            "b": b, "ns": n, "ok": rc == 0}
