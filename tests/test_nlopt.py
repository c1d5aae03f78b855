"""The NLopt Nelder-Mead restatement (deftri/nlopt_nm.py; NLopt absent and unpinned)
and deformationOptimization's weight search ("twoOptimizations" + "nlopt", the Simulation.yaml
default) on the CPU: NLopt's documented heuristics (default initial step, elimdim, bound pinning,
maxeval, xtol) on analytic objectives, then the outer loop with the oracle's arapOptimization.
Device parity of the outer loop is in test_gpu_parity.py::test_weight_search_matches_oracle."""
import math

import numpy as np
import pytest

from arap_oracle_fn import oracle_arap
from conftest import GOLDEN
from deftri import nlopt_nm, optimization

SIM_LB = [1.0, 50.0, 1e-5]            # Simulation.yaml:88-93
SIM_UB = [1.0, 50.0, 1e7]
SIM_X0 = [1.0, 50.0, 2e5]             # Optimization.rep / global / arap (:72-74)


def test_default_initial_step_heuristic():
    dx = nlopt_nm.default_initial_step(np.array([2e5]), np.array([1e-5]), np.array([1e7]))
    assert dx[0] == pytest.approx(0.75 * (2e5 - 1e-5))          # x - lb < (ub - lb) / 4
    dx = nlopt_nm.default_initial_step(np.array([9e6]), np.array([0.0]), np.array([1e7]))
    assert dx[0] == pytest.approx(0.75 * 1e6)                    # ub - x smallest
    dx = nlopt_nm.default_initial_step(np.array([5.0]), np.array([-math.inf]), np.array([math.inf]))
    assert dx[0] == 5.0                                          # unbounded: |x|
    dx = nlopt_nm.default_initial_step(np.array([0.0]), np.array([-math.inf]), np.array([math.inf]))
    assert dx[0] == 1.0


def test_elimdim_and_first_evaluations():
    seen = []

    def f(x):
        seen.append(np.array(x))
        return math.log(x[2] / 3e5) ** 2
    x, fmin, res, nev = nlopt_nm.nelder_mead(f, SIM_X0, SIM_LB, SIM_UB, 0.15, 0.15, 30)
    assert all(s[0] == 1.0 and s[1] == 50.0 for s in seen)      # lb == ub dimensions never move
    assert seen[0][2] == 2e5 and seen[1][2] == pytest.approx(2e5 + 0.75 * (2e5 - 1e-5))
    assert res in (nlopt_nm.XTOL_REACHED, nlopt_nm.MAXEVAL_REACHED) and nev == len(seen) <= 30
    assert abs(x[2] / 3e5 - 1) < 0.3 and fmin == min(f_ for f_ in (math.log(s[2] / 3e5) ** 2 for s in seen))


def test_quadratic_2d_converges_and_maxeval():
    f = lambda x: (x[0] - 1.5) ** 2 + 4 * (x[1] + 0.5) ** 2
    x, fmin, res, nev = nlopt_nm.nelder_mead(f, [0, 0], [-5, -5], [5, 5], 1e-8, 1e-10, 2000)
    assert res == nlopt_nm.XTOL_REACHED and np.allclose(x, [1.5, -0.5], atol=1e-6)
    x, fmin, res, nev = nlopt_nm.nelder_mead(f, [0, 0], [-5, -5], [5, 5], 1e-8, 1e-10, 7)
    assert res == nlopt_nm.MAXEVAL_REACHED and nev == 7


def test_bounds_pin_the_simplex():
    f = lambda x: (x[0] + 3.0) ** 2            # unconstrained optimum below lb
    x, fmin, res, nev = nlopt_nm.nelder_mead(f, [1.0], [0.0], [2.0], 1e-6, 1e-9, 200)
    assert x[0] == 0.0 and fmin == 9.0


def test_initial_guess_outside_bounds_rejected():
    with pytest.raises(ValueError):
        nlopt_nm.nelder_mead(lambda x: 0.0, [3.0], [0.0], [2.0])


def test_weight_search_outer_loop_on_oracle():
    """deformationOptimization with the Simulation.yaml selection (twoOptimizations + nlopt) on the
    reference's default 120-point scene, arapOptimization provided by the oracle."""
    import importlib
    import sys
    sys.path.insert(0, str(GOLDEN))
    mg = importlib.import_module("make_golden")
    m, st, sigma = mg.scene("sim_default")
    assert st.selection == "twoOptimizations" and st.weights_selection == "nlopt"
    st.depth_weight = 3.0                      # Simulation.yaml lacks DepthWeight
    st.n_optimizations, st.nlopt_iterations, st.n_iterations = 1, 6, 5
    rounds = optimization.deformationOptimization(m, st, arap_fn=oracle_arap)
    r = rounds[0]
    assert len(r["evaluations"]) == 6 and r["nlopt_result"] == nlopt_nm.MAXEVAL_REACHED
    assert r["evaluations"][0]["x"] == SIM_X0
    assert r["minf"] == min(e["f"] for e in r["evaluations"])
    assert r["weights"][:2] == [1.0, 50.0] and r["update"] > 0


@pytest.mark.parametrize("case", ["rosen2d", "quad3d_maxeval", "bounded1d", "sim_weights"])
def test_speculative_prefetch_matches_sequential(case):
    """nelder_mead(prefetch=...) evaluates the candidate points of each step in one batch (the
    multi-GPU weight search) and must reproduce the sequential run exactly: same x, minf, result,
    nevals and evaluation log."""
    f, x0, lb, ub, tr, ta, me = {
        "rosen2d": (lambda x: (1 - x[0]) ** 2 + 100 * (x[1] - x[0] ** 2) ** 2, [-1.2, 1.0], [-5, -5], [5, 5], 1e-10, 1e-12, 400),
        "quad3d_maxeval": (lambda x: (x[0] - 1) ** 2 + 2 * (x[1] + 2) ** 2 + 3 * x[2] ** 2, [0, 0, 1], [-4, -4, -4], [4, 4, 4], 0, 0, 57),
        "bounded1d": (lambda x: (x[0] + 3.0) ** 2, [1.0], [0.0], [2.0], 1e-6, 1e-9, 200),
        "sim_weights": (lambda x: math.log(x[2] / 3e5) ** 2 + 0.1 * math.sin(x[2] / 1e5), SIM_X0, SIM_LB, SIM_UB, 0.15, 0.15, 30),
    }[case]
    seq_log, spec_log, batches = [], [], []

    def prefetch(xs):
        batches.append(len(xs))
        return [f(x) for x in xs]
    a = nlopt_nm.nelder_mead(f, x0, lb, ub, tr, ta, me, log=seq_log.append)
    b = nlopt_nm.nelder_mead(f, x0, lb, ub, tr, ta, me, log=spec_log.append, prefetch=prefetch)
    assert np.array_equal(a[0], b[0]) and a[1:] == b[1:]
    assert seq_log == spec_log
    assert max(batches) > 1                                     # candidates really were batched


@pytest.mark.parametrize("case", ["rosen2d", "quad3d_maxeval", "bounded1d", "sim_weights", "fixed_dims", "shrink"])
def test_native_nelder_mead_matches_restatement(case):
    """The native restatement behind deftri_deformation_optimization (csrc/deformation.cpp, via
    deftri_debug_nelder_mead) and deftri/nlopt_nm.py are the same algorithm: the same evaluation
    sequence point for point, the same best point, minimum, result code and evaluation count."""
    from deftri import capi
    f, x0, lb, ub, tr, ta, me = {
        "rosen2d": (lambda x: (1 - x[0]) ** 2 + 100 * (x[1] - x[0] ** 2) ** 2, [-1.2, 1.0], [-5, -5], [5, 5], 1e-10, 1e-12, 400),
        "quad3d_maxeval": (lambda x: (x[0] - 1) ** 2 + 2 * (x[1] + 2) ** 2 + 3 * x[2] ** 2, [0, 0, 1], [-4, -4, -4], [4, 4, 4], 0, 0, 57),
        "bounded1d": (lambda x: (x[0] + 3.0) ** 2, [1.0], [0.0], [2.0], 1e-6, 1e-9, 200),
        "sim_weights": (lambda x: math.log(x[2] / 3e5) ** 2 + 0.1 * math.sin(x[2] / 1e5), SIM_X0, SIM_LB, SIM_UB, 0.15, 0.15, 30),
        "fixed_dims": (lambda x: (x[1] - 0.3) ** 2 + abs(x[2]), [1.0, 0.0, 2.0], [1.0, -1.0, -3.0], [1.0, 1.0, 3.0], 1e-7, 1e-9, 300),
        "shrink": (lambda x: abs(x[0]) + abs(x[1]) + 0.01 * x[0] * x[1], [2.0, -1.5], [-4, -4], [4, 4], 1e-9, 1e-12, 500),
    }[case]
    seq = []
    a = nlopt_nm.nelder_mead(f, x0, lb, ub, tr, ta, me, log=seq.append)
    x, minf, res, nev, seen = capi.nelder_mead_native(f, x0, lb, ub, tr, ta, me)
    assert [e["x"] for e in seq] == seen
    assert list(a[0]) == x and a[1] == minf and a[2] == res and a[3] == nev


def test_global_insert_is_the_map_models():
    """Map::insertGlobalKeyFramesTransformation's two entries (deftri_global_insert): the Map model
    stores exactly what the native loop stores, the inverse entry composes with the forward one to
    the identity within fp32 rounding, and both are unit quaternions with w >= 0."""
    from deftri import capi
    from deftri.mapmodel import Map, SE3f, mat_from_quat
    t7 = [0.01, -0.02, 0.03, 0.999, 0.004, -0.002, 0.001]
    fwd, inv = capi.global_insert(t7)
    m = Map()
    m.insert_global_from7(0, 1, t7)
    assert list(m.global_T[(0, 1)].as7()) == fwd and list(m.global_T[(1, 0)].as7()) == inv
    for q in (fwd[:4], inv[:4]):
        assert abs(np.linalg.norm(q) - 1) < 1e-15 and q[3] >= 0
    Ra, Rb = mat_from_quat(fwd[:4]), mat_from_quat(inv[:4])
    assert np.allclose(Ra @ Rb, np.eye(3), atol=1e-6)
    assert np.allclose(Ra @ np.array(inv[4:]) + np.array(fwd[4:]), 0, atol=1e-6)
