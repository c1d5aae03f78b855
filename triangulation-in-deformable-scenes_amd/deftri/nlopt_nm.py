"""Nelder–Mead weight search of the reference's outer loop.

The reference's `deformationOptimization` (g2oBundleAdjustment.cc:486-530, the Simulation.yaml
default `selection: twoOptimizations`, `weightsSelection: nlopt`) runs

    nlopt::opt opt(nlopt::LN_NELDERMEAD, 3);  set_lower_bounds / set_upper_bounds;
    set_min_objective(outerObjective);  set_xtol_rel; set_xtol_abs; set_maxeval;  optimize(x, minf)

NLopt is a third-party dependency absent from /root/reference (no vendored copy, no lock file:
version unpinned).  This module restates NLopt 2.x's published algorithm for that call
(`src/algs/neldermead/nldrmd.c`, `nlopt_set_default_initial_step`, the `elimdim` wrapper that
removes dimensions with lb == ub, and the `relstop` stopping tests) as host logic: every objective
evaluation is a device `arapOptimization` on a map clone (deftri/optimization.py).

  simplex        x0 and x0 + dx_i e_i (dx from the default-step heuristic), pinned into the bounds
  ordering       by f, ties by position in the point table (NLopt's red-black tree key)
  step           reflect (alpha 1) the worst point through the centroid of the others; expand
                 (gamma 2) on a new best; accept if better than the second worst; otherwise
                 contract (beta 0.5, inside if f(xr) >= f(xh)); on a failed contraction shrink
                 (delta 0.5) towards the best point.  Every new point is pinned into [lb, ub].
  stop           x: every coordinate of the simplex's radius around the centroid within
                 max(xtol_abs, xtol_rel * |x|); coincident reflected point; maxeval
"""
import math

import numpy as np

ALPHA, BETA, GAMMA, DELTA = 1.0, 0.5, 2.0, 0.5

SUCCESS, FTOL_REACHED, XTOL_REACHED, MAXEVAL_REACHED, FAILURE = 1, 3, 4, 5, -1


def default_initial_step(x, lb, ub):
    """nlopt_set_default_initial_step: crude per-dimension step from the bounds and x."""
    dx = np.zeros(len(x))
    for i in range(len(x)):
        step = math.inf
        if math.isfinite(ub[i]) and math.isfinite(lb[i]) and (ub[i] - lb[i]) * 0.25 < step and ub[i] > lb[i]:
            step = (ub[i] - lb[i]) * 0.25
        if math.isfinite(ub[i]) and ub[i] - x[i] < step and ub[i] > x[i]:
            step = (ub[i] - x[i]) * 0.75
        if math.isfinite(lb[i]) and x[i] - lb[i] < step and x[i] > lb[i]:
            step = (x[i] - lb[i]) * 0.75
        if math.isinf(step):
            if math.isfinite(ub[i]) and abs(ub[i] - x[i]) < abs(step):
                step = (ub[i] - x[i]) * 1.1
            if math.isfinite(lb[i]) and abs(x[i] - lb[i]) < abs(step):
                step = (x[i] - lb[i]) * 1.1
        if math.isinf(step) or abs(step) < 1e-300:
            step = x[i]
        if math.isinf(step) or step == 0.0:
            step = 1.0
        dx[i] = step
    return dx


def _close(a, b):
    return abs(a - b) <= 1e-13 * (abs(a) + abs(b))


def _relstop(vold, vnew, reltol, abstol):
    if math.isinf(vold):
        return False
    d = abs(vnew - vold)
    return d < abstol or d < reltol * (abs(vnew) + abs(vold)) * 0.5 or (reltol > 0 and vnew == vold)


def _reflect(c, scale, xold, lb, ub):
    """xnew = c + scale (c - xold) pinned to the bounds; None when xnew coincides with c or xold."""
    xnew = c + scale * (c - xold)
    xnew = np.minimum(np.maximum(xnew, lb), ub)
    equalc = all(_close(xnew[i], c[i]) for i in range(len(c)))
    equalold = all(_close(xnew[i], xold[i]) for i in range(len(c)))
    return None if (equalc or equalold) else xnew


def _simplex_vertex(x, xstep, lo, hi, i):
    """Initial simplex vertex i of nldrmd_minimize (x + xstep_i e_i, kept inside the bounds)."""
    pt = x.copy()
    pt[i] += xstep[i]
    if pt[i] > hi[i]:
        pt[i] = hi[i] if hi[i] - x[i] > abs(xstep[i]) * 0.1 else x[i] - abs(xstep[i])
    if pt[i] < lo[i]:
        if x[i] - lo[i] > abs(xstep[i]) * 0.1:
            pt[i] = lo[i]
        else:
            pt[i] = x[i] + abs(xstep[i])
            if pt[i] > hi[i]:
                pt[i] = 0.5 * ((hi[i] if hi[i] - x[i] > x[i] - lo[i] else lo[i]) + x[i])
    return pt


class _Stop(Exception):
    def __init__(self, code):
        super().__init__(code)
        self.code = code


def nelder_mead(f, x0, lb, ub, xtol_rel=0.0, xtol_abs=0.0, maxeval=0, log=None, prefetch=None):
    """opt.optimize(x, minf) of an LN_NELDERMEAD nlopt::opt.  Returns (x, minf, result, nevals).

    prefetch (optional): callable(list of full x) -> list of f values, called with every point the
    next sequential step may evaluate (the initial simplex; reflection, expansion and both
    contractions; the shrink points), so a caller can evaluate them concurrently (e.g. one LM solve
    per GPU).  The algorithm then consumes the values in NLopt's order: results, the evaluation
    log and nevals are those of the sequential run; points NLopt would not have evaluated are
    computed and discarded."""
    x0 = np.asarray(x0, np.float64)
    lb = np.asarray(lb, np.float64)
    ub = np.asarray(ub, np.float64)
    if np.any(x0 < lb) or np.any(x0 > ub):
        raise ValueError("initial guess outside of bounds (nlopt NLOPT_INVALID_ARGS)")
    # elimdim: dimensions with lb == ub are fixed and removed from the search
    free = np.nonzero(lb != ub)[0]
    xfull = x0.copy()
    state = {"nevals": 0, "minf": math.inf, "x": x0.copy()}
    cache = {}

    def full(xr):
        xf = xfull.copy()
        xf[free] = xr
        return xf

    def spec(points):
        if prefetch is None:
            return
        todo = []
        for xr in points:
            if xr is None:
                continue
            k = tuple(full(xr).tolist())
            if k not in cache and k not in [tuple(t.tolist()) for t in todo]:
                todo.append(full(xr))
        if todo:
            for xf, v in zip(todo, prefetch(todo)):
                cache[tuple(xf.tolist())] = float(v)

    def feval(xr):
        xf = full(xr)
        k = tuple(xf.tolist())
        v = cache.pop(k) if k in cache else float(f(xf))
        state["nevals"] += 1
        if log:
            log({"eval": state["nevals"], "x": xf.tolist(), "f": v})
        return v

    def check(xr, fv):          # CHECK_EVAL
        if fv <= state["minf"]:
            state["minf"] = fv
            xf = xfull.copy()
            xf[free] = xr
            state["x"] = xf
        if maxeval > 0 and state["nevals"] >= maxeval:
            raise _Stop(MAXEVAL_REACHED)

    n = len(free)
    x = x0[free].copy()
    try:
        if n == 0:
            check(x, feval(x))
            return state["x"], state["minf"], SUCCESS, state["nevals"]
        lo, hi = lb[free], ub[free]
        xstep = default_initial_step(x, lo, hi)
        spec([x] + [_simplex_vertex(x, xstep, lo, hi, i) for i in range(n)])
        fx = feval(x)                                                   # nldrmd_minimize: f(x0) first
        check(x, fx)
        pts = np.zeros((n + 1, n))
        fv = np.zeros(n + 1)
        pts[0] = x
        fv[0] = fx
        for i in range(n):
            pt = _simplex_vertex(x, xstep, lo, hi, i)
            if _close(pt[i], x[i]):
                raise _Stop(FAILURE)
            pts[i + 1] = pt
            fv[i + 1] = feval(pt)
            check(pt, fv[i + 1])
        while True:
            order = sorted(range(n + 1), key=lambda k: (fv[k], k))       # rb-tree: f, then address
            il, ih = order[0], order[-1]
            fl, fh = fv[il], fv[ih]
            xl, xh = pts[il].copy(), pts[ih].copy()
            c = np.zeros(n)
            for k in range(n + 1):
                if k != ih:
                    c += pts[k]
            c *= 1.0 / n
            xcur = np.max(np.abs(pts - c), axis=0) + c
            if all(_relstop(xcur[i], c[i], xtol_rel, xtol_abs) for i in range(n)):
                raise _Stop(XTOL_REACHED)
            xr = _reflect(c, ALPHA, xh, lo, hi)
            if xr is None:
                raise _Stop(XTOL_REACHED)
            spec([xr, _reflect(c, GAMMA, xh, lo, hi), _reflect(c, -BETA, xh, lo, hi), _reflect(c, BETA, xh, lo, hi)])
            fr = feval(xr)
            check(xr, fr)
            if fr < fl:                                                 # new best: expand
                xe = _reflect(c, GAMMA, xh, lo, hi)
                if xe is None:
                    raise _Stop(XTOL_REACHED)
                fe = feval(xe)
                check(xe, fe)
                if fe >= fr:
                    pts[ih], fv[ih] = xr, fr
                else:
                    pts[ih], fv[ih] = xe, fe
            elif fr < fv[order[-2]]:                                    # accept
                pts[ih], fv[ih] = xr, fr
            else:                                                       # contract
                xc = _reflect(c, -BETA if fh <= fr else BETA, xh, lo, hi)
                if xc is None:
                    raise _Stop(XTOL_REACHED)
                fc = feval(xc)
                check(xc, fc)
                if fc < fr and fc < fh:
                    pts[ih], fv[ih] = xc, fc
                else:                                                   # shrink towards the best
                    spec([_reflect(xl, -DELTA, pts[k], lo, hi) for k in range(n + 1) if k != il])
                    for k in range(n + 1):
                        if k == il:
                            continue
                        xs = _reflect(xl, -DELTA, pts[k], lo, hi)
                        if xs is None:
                            raise _Stop(XTOL_REACHED)
                        pts[k] = xs
                        fv[k] = feval(xs)
                        check(xs, fv[k])
    except _Stop as s:
        return state["x"], state["minf"], s.code, state["nevals"]
