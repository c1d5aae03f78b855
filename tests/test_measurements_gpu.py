"""§8 f3 — Measurements.cc on the device (deftri_measure_sim_absolute_map_errors,
deftri_measure_relative_map_errors) against the host restatement (tests/measurements_ref.py), on the
golden scenes (the reference's data files) before and after the device arapOptimization, at C2 size
and on a 3-keyframe map with a stored global transformation.  Counts exact; the device sums in
double in a fixed tree where the reference accumulates absolute errors in float sequentially
(relative 1e-5 covers the float accumulation at 1e5 terms) and relative errors in double (1e-9)."""
import numpy as np
import pytest

from conftest import GOLDEN
from deftri import metrics, optimization, sim
from measurements_ref import relative, sim_absolute

pytestmark = pytest.mark.gpu


def _check_abs(m, orig, moved, rtol):
    got = metrics.measureSimAbsoluteMapErrors(m, orig, moved)
    ref = sim_absolute(m, orig, moved)
    assert got["point_count"] == ref["point_count"]
    for k in ("average_movement", "average_error_original", "average_error_moved", "average_error", "rmse"):
        assert got[k] == pytest.approx(ref[k], rel=rtol), k


def _check_rel(m):
    got = metrics.measureRelativeMapErrors(m)
    ref = relative(m)
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        for k in ("kf1", "kf2", "reported", "valid_pairs", "n_matches"):
            assert g[k] == r[k], k
        for k in ("rel_error", "depth_error", "global_t_error", "area"):
            assert g[k] == pytest.approx(r[k], rel=1e-9, abs=1e-300), k


def test_golden_scenes_before_and_after_arap(golden_cases):
    import importlib, sys
    sys.path.insert(0, str(GOLDEN))
    mg = importlib.import_module("make_golden")
    for name in golden_cases:
        m, st, sigma = mg.scene(name)
        orig, moved, _ = mg.case_inputs(name)
        _check_abs(m, orig, moved, 1e-6)
        _check_rel(m)
        optimization.arapOptimization(m, st.rep, st.global_, st.arap, st.alpha, st.beta, sigma, 10)
        _check_abs(m, orig, moved, 1e-6)
        _check_rel(m)


def test_c2_size():
    m, gt = sim.simulate_two_view(n=100000, seed=1, scale_scene=True, compact=True)
    _check_abs(m, gt["original"], gt["moved"], 1e-5)
    _check_rel(m)


def test_multi_keyframe_with_global_transform():
    from deftri.mapmodel import SE3f, mat_from_quat
    m, gt = sim.simulate_multi_view(n=300, k=3, seed=12)
    q = np.array([0.01, 0.02, -0.015, 1.0]); q /= np.linalg.norm(q)
    m.insert_global_T(0, 1, SE3f(mat_from_quat(q).astype(np.float32), np.array([0.002, 0.001, -0.003], np.float32)))
    _check_rel(m)
