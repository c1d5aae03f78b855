"""Headline workload parity (C2: 100k correspondences x 2 views, bench.py's scene) against the
committed oracle run (tests/golden/c2, tests/golden/make_c2_golden.py: the reference LM restated in
C with g2o numeric Jacobians — the reference's arithmetic — on the same full-size graph, 6 LM
iterations).  The device runs the same iterations in the same numeric mode on BOTH plans — the
iterative plan's tile chain is the one bench.py times (600,008 unknowns) — : identical trial counts,
chi2 per iteration within the band derived from the oracle's own order spread (below), the solved
points (fixed subsample and coordinate sums) and the reprojection RMSE of the solved map
(calculatePixelsStandDev) within the north-star 1e-4 px.  (This near-stalled headline LM moves the
RMSE by ~1e-4 px; tests/test_regime_goldens.py pins the merged chain at 30k correspondences on runs
whose RMSE moves by > 5e-3 px.)

c2_realcolon: the same 100k scene under Data/Realcolon.yaml's weights and distorted KB8 camera
(rep 1, arap 0.1, sigma_d 1e-6 m), 20 oracle iterations: chi2 falls by 9 orders of magnitude (the
depth edges dominate), the RMSE moves by 7e-4 px — 7x the 1e-4 px tolerance — and the tile chain
(the plan bench.py times) must land on the oracle's solution.

ns500k_realcolon: the north-star size (500k correspondences x 2 views, 3,000,008 unknowns) under the
same weights, 4 oracle iterations (tests/golden/make_c2_golden.py realcolon 4 500000), on the tile
chain only."""
import copy
import json

import numpy as np
import pytest

from conftest import GOLDEN
from deftri import capi, metrics, sim

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["c2", "c2_realcolon", "ns500k_realcolon"])
def golden(request):
    d = GOLDEN / request.param
    if not (d / "expected_c2.json").exists():
        pytest.skip("C2 golden not generated")
    return json.loads((d / "expected_c2.json").read_text()), np.load(d / "expected_c2.npz")


@pytest.fixture(scope="module")
def c2_scene(golden):
    meta, _ = golden
    w = meta.get("weights")
    if w is None or meta.get("regime", "simulation") == "simulation":
        return sim.two_view_problem(meta["n_corr"], meta["seed"], return_map=True)
    return sim.two_view_problem(meta["n_corr"], meta["seed"], w["rep"], w["arap"], np.float32(w["depth_sigma"]),
                                return_map=True, kb8=getattr(sim, w["camera"]))


@pytest.mark.parametrize("plan", ["iterative", "multifrontal"])
def test_c2_iterations_match_oracle(gpu_ctx, golden, c2_scene, plan):
    meta, z = golden
    if plan == "multifrontal" and meta["n_corr"] > 100000:
        pytest.skip("the north-star golden pins the timed (iterative) plan")
    p, m0 = c2_scene
    m = copy.deepcopy(m0)
    assert p.summary() == meta["summary"]
    if "problem_digest" in meta:                      # the graph the golden was computed on
        assert p.digest() == meta["problem_digest"], "stale golden: the graph builder changed the graph"
    gpu_ctx.set_plan(plan)
    try:
        gpu_ctx.set_lm_lanes(1)
        gpu_ctx.upload(p)
        info = gpu_ctx.plan_info()
        assert info["plan"] == plan
        if plan == "iterative":
            assert info["tiles"] > 0 and info["cg_launches"] in (1, 2)   # the tile chain bench.py times
        r = gpu_ctx.solve_lm(meta["n_iterations"], analytic=False)
        pts, sc, tg = gpu_ctx.download()
    finally:
        gpu_ctx.set_plan("multifrontal")
        gpu_ctx.set_lm_lanes(0)
    if plan == "iterative":
        assert r["pcg_trials"] == r["trials_total"] and r["pcg_fallbacks"] == 0
    assert r["chi2_initial"] == pytest.approx(meta["chi2_initial"], rel=1e-11)
    assert r["iterations"] == meta["iterations"]
    assert r["trials_iter"] == list(z["trials_iter"])
    # chi2 per iteration within max(4 x the oracle's own spread between elimination orders, 1e-6), the
    # rule of tests/test_regime_goldens.py: the spread recorded in the golden's oracle_order_spread
    # (tools/oracle_spread.py; the Simulation C2 run is well conditioned and has none: 1e-6).  Under
    # Realcolon's weights (Omega_depth 1e12) iteration 9 is conditioning-bound: with the SE3 / depth
    # arithmetic uncontracted as in the reference (device_math.h) both device plans land 9.3-9.4e-7 from
    # the oracle (2.3e-6 with FMA contraction); the oracle itself moves 2.6e-6 there when its edge sums
    # run backwards (the recorded spread).
    spread = meta.get("oracle_order_spread", {}).get("max_rel_chi2", 0.0)
    tol = max(4.0 * spread, 1e-6)
    dev = np.abs(np.asarray(r["chi2_iter"]) - z["chi2_iter"]) / np.abs(z["chi2_iter"])
    print(f"{meta.get('regime', 'simulation')}/{plan}: chi2 max rel dev {dev.max():.3e} at {int(dev.argmax())}, "
          f"oracle order spread {spread:.3e}, tolerance {tol:.3e}")
    assert dev.max() <= tol, (dev.max(), int(dev.argmax()), tol)
    # the final damping inherits the chi2 deviations through g2o's rho rule (a ratio of chi2
    # differences): the same rule, 4 x the oracle's own spread of lambda_final (recorded with the chi2
    # spread), 1e-9 where none is recorded
    lam_tol = max(4.0 * meta.get("oracle_order_spread", {}).get("max_rel_lambda", 0.0), 1e-9)
    assert r["lambda_final"] == pytest.approx(meta["lambda_final"], rel=lam_tol)
    if meta.get("regime") == "realcolon" and meta["n_corr"] == 100000:   # the pin is meaningful: the
        assert abs(meta["rms_final"]["desv"] - meta["rms_initial"]["desv"]) > 5e-4   # solve moves the RMSE
    if meta["n_corr"] > 100000:                       # north-star size, 4 iterations: chi2 falls 1500x
        assert meta["chi2_final"] < 1e-3 * meta["chi2_initial"]
    ext = np.abs(pts).max()
    assert np.abs(pts[::meta["stride"]] - z["points_sub"]).max() <= 1e-7 * ext
    np.testing.assert_allclose(pts.sum(0), meta["point_sum"], rtol=1e-9)
    np.testing.assert_allclose(sc, meta["scales"], rtol=1e-7)
    metrics.apply_solution(m, list(p.point_ids), pts)
    rms = metrics.pixels_stand_dev(m)
    assert abs(rms["desv"] - meta["rms_final"]["desv"]) < 1e-4
    assert abs(rms["desvc1"] - meta["rms_final"]["desvc1"]) < 1e-4
    assert abs(rms["desvc2"] - meta["rms_final"]["desvc2"]) < 1e-4
