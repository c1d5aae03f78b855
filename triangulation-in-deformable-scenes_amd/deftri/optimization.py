"""Mirror of the reference's optimization API (Modules/Optimization/g2oBundleAdjustment.h:36-75)
over the C-ABI.  Same names, argument meaning and write-back behaviour:

  arapOptimization(pMap, rep, global, arap, alpha, beta, depthError, nIt, optimizationUpdate)
      builds the graph (host C++), runs g2o-semantics LM on the GPU, writes back fp32 positions,
      depth scales and the global KF-pair transformation; returns sum ||p_old - p_new||
      (g2oBundleAdjustment.cc:608-1008).
  deformationOptimization(pMap, settings, originalPoints, movedPoints)
      outer rounds until sum ||dp|| < 1e-4 * |MapPoints| (:446-606): fixed weights ("g2oArap") or
      the NLopt Nelder-Mead weight search ("twoOptimizations" + "nlopt", deftri/nlopt_nm.py) whose
      every evaluation is an arapOptimization on a map clone (outerObjective,
      nloptOptimization.cc:5-38).
  bundleAdjustment / localBundleAdjustment / poseOnlyOptimization
      BA entry points (no callers at the reference's HEAD): the BlockSolver_6_3 Schur
      LM on the device (deftri/ba.py over deftri_ba_*).
"""
import threading

from . import capi

_tls = threading.local()


def _ctx(device=0):
    c = getattr(_tls, "ctx", None)
    if c is None or c.device != device:
        c = capi.Context(device)
        _tls.ctx = c
    return c


def arapOptimization(pMap, repBalanceWeight, globalBalanceWeight, arapBalanceWeight, alphaWeight,
                     betaWeight, DepthError, nOptIterations, optimizationUpdate=None, device=0,
                     report=None):
    """Returns the optimization update (sum of point displacements); if `optimizationUpdate` is a
    one-element list it is written like the reference's out-parameter."""
    upd, rep = _ctx(device).arap_optimization(pMap, repBalanceWeight, globalBalanceWeight, arapBalanceWeight,
                                              alphaWeight, betaWeight, DepthError, nOptIterations)
    if isinstance(optimizationUpdate, list):
        if optimizationUpdate:
            optimizationUpdate[0] = upd
        else:
            optimizationUpdate.append(upd)
    if isinstance(report, dict):
        report.update(rep)
    return upd


def outerObjective(x, pMap, settings, arap_fn=None, device=0):
    """nloptOptimization.cc:5-38: arapOptimization on a clone of the map with weights x = (rep,
    global, arap), then (log desvc1)^2 + (log desvc2)^2 of calculatePixelsStandDev."""
    from . import metrics
    clone = pMap.clone()                        # pData->pMap->clone()
    fn = arap_fn or (lambda m, *a: arapOptimization(m, *a, device=device))
    fn(clone, float(x[0]), float(x[1]), float(x[2]), settings.alpha, settings.beta, settings.depth_sigma,
       settings.n_iterations)
    # calculatePixelsStandDev: on the device (deftri_pixels_stand_dev); the host restatement only
    # when a test substitutes the solver (arap_fn)
    pe = metrics.pixels_stand_dev(clone) if arap_fn is not None else _ctx(device).pixels_stand_dev(clone)

    return _log2(pe["desvc1"]) + _log2(pe["desvc2"])


def _log2(v):
    """std::pow(std::log(v), 2) (nloptOptimization.cc:31-32): +inf at 0, NaN below 0 or for NaN."""
    import math
    if v != v or v < 0:
        return math.nan
    return math.inf if v == 0 else math.log(v) ** 2


def deformationOptimization(pMap, settings, originalPoints=None, movedPoints=None, device=0, log=None,
                            arap_fn=None, workers=None, native=True):
    """g2oBundleAdjustment.cc:446-606.  Outer rounds until sum ||dp|| < 1e-4 |MapPoints| or
    numberOfOptimizations; per round either the fixed weights ("g2oArap") or the weight search
    ("twoOptimizations" + "nlopt": Nelder-Mead over (rep, global, arap) within the nlopt bounds,
    each evaluation an arapOptimization on a map clone, then arapOptimization on the map with the
    optimum, which becomes the next round's start).

    native (default): the whole loop behind the C-ABI (deftri_deformation_optimization: the search
    restated in C++, clones of the map's positions / scales / global table, every evaluation on the
    device), one call.  native=False: this host loop over deftri/nlopt_nm.py — the same algorithm
    (tests hold the two to the same search path).  `arap_fn` (tests only) replaces the device
    arapOptimization with another implementation of the same signature; `workers`
    (deftri.workers.ObjectiveWorkers) evaluates each Nelder-Mead step's candidate points on several
    GPUs at once (the search and its result are those of the sequential run); both use the host loop."""
    from .nlopt_nm import nelder_mead
    settings.validate_for_solver()
    if native and arap_fn is None and workers is None:
        r = _ctx(device).deformation_optimization(pMap, settings)
        rounds = []
        for k in range(r["rounds"]):
            info = {"round": k + 1, "weights": r["round_weights"][k] if k < 64 else r["weights"],
                    "update": r["round_update"][k] if k < 64 else r["update"],
                    "evaluations": [e for e in r["evaluations"] if e["round"] == k + 1]}
            if k == r["rounds"] - 1 and settings.selection == "twoOptimizations" and settings.weights_selection == "nlopt":
                info.update({"minf": r["minf"], "nlopt_result": r["nlopt_result"]})
            rounds.append(info)
            if log:
                log(info)
        return rounds
    if settings.selection == "open3DArap":
        raise NotImplementedError("open3DArap is a different algorithm (Open3D DeformAsRigidAsPossible), out of scope")
    # weightsSelection other than "nlopt" (the Eigen LM, :531-564): Eigen::LevenbergMarquardt::minimize
    # returns ImproperInputParameters before any evaluation (the functor declares 2 values for the 3
    # weights, m < n, EigenOptimization.h:31), so the round is arapOptimization at the unchanged weights
    search = settings.selection == "twoOptimizations" and settings.weights_selection == "nlopt"

    def run_arap(m, rep, glob, arap):
        if arap_fn is not None:
            return arap_fn(m, rep, glob, arap, settings.alpha, settings.beta, settings.depth_sigma,
                           settings.n_iterations)
        return arapOptimization(m, rep, glob, arap, settings.alpha, settings.beta, settings.depth_sigma,
                                settings.n_iterations, device=device)

    n_mp = len(pMap.map_points)
    rep_w, glob_w, arap_w = settings.rep, settings.global_, settings.arap
    update = 100.0
    rounds = []
    i = 1
    while i <= settings.n_optimizations and update >= 0.0001 * n_mp:
        info = {"round": i}
        if search:
            base = pMap.clone()                   # optData.pMap = pMap->clone()
            evals = []
            prefetch = None
            if workers is not None and arap_fn is None:
                prefetch = lambda xs, base=base: workers.map_objective(xs, base, settings)
            x, minf, res, nev = nelder_mead(
                lambda x: outerObjective(x, base, settings, arap_fn=arap_fn, device=device),
                [rep_w, glob_w, arap_w],
                [settings.nlopt_rep_lb, settings.nlopt_global_lb, settings.nlopt_arap_lb],
                [settings.nlopt_rep_ub, settings.nlopt_global_ub, settings.nlopt_arap_ub],
                xtol_rel=settings.nlopt_rel_tol, xtol_abs=settings.nlopt_abs_tol,
                maxeval=int(settings.nlopt_iterations), log=evals.append, prefetch=prefetch)
            if res < 0:        # nlopt::opt::optimize throws on a failure code (before :525)
                raise RuntimeError(f"nlopt failure (result {res}) in round {i}")
            rep_w, glob_w, arap_w = (float(v) for v in x)
            info.update({"weights": [rep_w, glob_w, arap_w], "minf": minf, "nlopt_result": res,
                         "evaluations": evals})
        update = run_arap(pMap, rep_w, glob_w, arap_w)
        info["update"] = update
        rounds.append(info)
        if log:
            log(info)
        i += 1
    return rounds


def bundleAdjustment(pMap, device=0, report=None):
    """g2oBundleAdjustment.cc:38-138 on the device BA path (deftri/ba.py)."""
    from . import ba
    return ba.bundleAdjustment(pMap, device=device, report=report)


def localBundleAdjustment(pMap, currKeyFrameId, device=0, report=None):
    """g2oBundleAdjustment.cc:245-444 on the device BA path (deftri/ba.py)."""
    from . import ba
    return ba.localBundleAdjustment(pMap, currKeyFrameId, device=device, report=report)


def poseOnlyOptimization(currFrame, device=0, report=None):
    """g2oBundleAdjustment.cc:140-243 on the device BA path (deftri/ba.py); returns the inlier count."""
    from . import ba
    return ba.poseOnlyOptimization(currFrame, device=device, report=report)
