"""Mirror of the reference's optimization API (Modules/Optimization/g2oBundleAdjustment.h:36-75)
over the C-ABI.  Same names, argument meaning and write-back behaviour:

  arapOptimization(pMap, rep, global, arap, alpha, beta, depthError, nIt, optimizationUpdate)
      builds the graph (host C++), runs g2o-semantics LM on the GPU, writes back fp32 positions,
      depth scales and the global KF-pair transformation; returns sum ||p_old - p_new||
      (g2oBundleAdjustment.cc:608-1008).
  deformationOptimization(pMap, settings, originalPoints, movedPoints)
      outer rounds until sum ||dp|| < 1e-4 * |MapPoints| (:446-606) with fixed weights
      ("g2oArap" selection).  The NLopt / Eigen weight tuning of "twoOptimizations" is the next
      component and raises NotImplementedError here.
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


def deformationOptimization(pMap, settings, originalPoints=None, movedPoints=None, device=0, log=None):
    settings.validate_for_solver()
    if settings.selection == "twoOptimizations":
        raise NotImplementedError("twoOptimizations (NLopt/Eigen weight tuning) is the next component; "
                                  "use selection 'g2oArap' (fixed weights)")
    if settings.selection == "open3DArap":
        raise NotImplementedError("open3DArap is a different algorithm (Open3D DeformAsRigidAsPossible), out of scope")
    n_mp = len(pMap.map_points)
    update = 100.0
    rounds = []
    i = 1
    while i <= settings.n_optimizations and update >= 0.0001 * n_mp:
        rep = {}
        update = arapOptimization(pMap, settings.rep, settings.global_, settings.arap, settings.alpha,
                                  settings.beta, settings.depth_sigma, settings.n_iterations, device=device,
                                  report=rep)
        rounds.append({"round": i, "update": update, "chi2_final": rep.get("chi2_final")})
        if log:
            log(rounds[-1])
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
