"""Headline workload parity (C2: 100k correspondences x 2 views, bench.py's scene) against the
committed oracle run (tests/golden/c2, tests/golden/make_c2_golden.py: the reference LM restated in
C with g2o numeric Jacobians — the reference's arithmetic — on the same full-size graph).  The
device runs the same first iterations in the same numeric mode; identical trial counts, chi2 per
iteration rel 1e-6, the solved points (fixed subsample and coordinate sums) and the reprojection
RMSE of the solved map (calculatePixelsStandDev) within the north-star 1e-4 px."""
import json

import numpy as np
import pytest

from conftest import GOLDEN
from deftri import capi, metrics, sim

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def golden():
    d = GOLDEN / "c2"
    if not (d / "expected_c2.json").exists():
        pytest.skip("C2 golden not generated")
    return json.loads((d / "expected_c2.json").read_text()), np.load(d / "expected_c2.npz")


def test_c2_first_iterations_match_oracle(gpu_ctx, golden):
    meta, z = golden
    p, m = sim.two_view_problem(meta["n_corr"], meta["seed"], return_map=True)
    assert p.summary() == meta["summary"]
    gpu_ctx.set_lm_lanes(1)
    gpu_ctx.upload(p)
    r = gpu_ctx.solve_lm(meta["n_iterations"], analytic=False)
    gpu_ctx.set_lm_lanes(0)
    assert r["chi2_initial"] == pytest.approx(meta["chi2_initial"], rel=1e-11)
    assert r["iterations"] == meta["iterations"]
    assert r["trials_iter"] == list(z["trials_iter"])
    np.testing.assert_allclose(r["chi2_iter"], z["chi2_iter"], rtol=1e-6)
    assert r["lambda_final"] == pytest.approx(meta["lambda_final"], rel=1e-9)
    pts, sc, tg = gpu_ctx.download()
    ext = np.abs(pts).max()
    assert np.abs(pts[::meta["stride"]] - z["points_sub"]).max() <= 1e-7 * ext
    np.testing.assert_allclose(pts.sum(0), meta["point_sum"], rtol=1e-9)
    np.testing.assert_allclose(sc, meta["scales"], rtol=1e-7)
    metrics.apply_solution(m, list(p.point_ids), pts)
    rms = metrics.pixels_stand_dev(m)
    assert abs(rms["desv"] - meta["rms_final"]["desv"]) < 1e-4
    assert abs(rms["desvc1"] - meta["rms_final"]["desvc1"]) < 1e-4
    assert abs(rms["desvc2"] - meta["rms_final"]["desvc2"]) < 1e-4
