"""Full-size properties of the timed plan (the iterative plan, merged two-launch CG chain) at the
BASELINE sizes, where the oracle takes minutes to hours per iteration: properties that hold for any
correct g2o LM (g2oBundleAdjustment.cc:959-962) and need no reference run.

  * accepted chi2 never increases (an LM iteration keeps only a trial with rho > 0)
  * no PCG step fails (every trial solved by PCG within its budget)
  * a repeated run from the same state is bit-identical (fixed-order sums, no atomics)
  * a damped solve (H + lambda I) x = b at the LM's dampings has a true relative residual
    ||b - (H + lambda I) x|| / ||b|| < 1e-11, measured with the plan's own matrix-free product
    (deftri_eval_hessian_product on the iterative plan; the CG stops on its recurrence residual at
    1e-12), and a normwise backward error ||r|| / (||(H + lambda I) x|| + ||b||) < 1e-12

C2: bench.py's headline scene (100k correspondences x 2 views, 600,008 unknowns).  C3 shape: 50k
correspondences x 8 keyframes, all 28 pairs (1.2M unknowns, 8.4M ARAP edges; Drunkard.yaml shapes
and weights), bench.py --workload c3's scene.  C4: 500k x 8 keyframes, all 28 pairs (12M unknowns,
84M ARAP edges), bench.py --workload c4's scene."""
import numpy as np
import pytest

from deftri import capi, sim

pytestmark = pytest.mark.gpu


def c2_problem():
    return sim.two_view_problem(100000, 1)            # bench.py build_problem(100000, 1)


def c4_problem():
    return sim.multi_view_problem(500000, 8, seed=1, kb8=sim.DRUNKARD_KB8, rep_weight=1.0, arap_weight=1e7,
                                  depth_sigma=np.float32(0.3), pair_window=0)


def c3_problem():
    return sim.multi_view_problem(50000, 8, seed=1, kb8=sim.DRUNKARD_KB8, rep_weight=1.0, arap_weight=1e7,
                                  depth_sigma=np.float32(0.3), pair_window=0)


def check_props(p, n_it, lambdas_rel):
    with capi.Context(0) as ctx:
        ctx.set_plan("auto")                      # the library's choice: iterative from 50k unknowns
        ctx.upload(p)
        info = ctx.plan_info()
        assert info["plan"] == "iterative" and info["cg_launches"] in (1, 2)   # tile (C2) or merged chain
        r1 = ctx.solve_lm(n_it, analytic=False)
        s1 = ctx.download()
        assert r1["iterations"] == n_it
        assert r1["pcg_fallbacks"] == 0 and r1["pcg_trials"] == r1["trials_total"]
        chi = [r1["chi2_initial"]] + list(r1["chi2_iter"])
        assert all(b <= a for a, b in zip(chi, chi[1:])), chi
        assert r1["chi2_final"] < r1["chi2_initial"]
        ctx.reset_state()
        r2 = ctx.solve_lm(n_it, analytic=False)
        s2 = ctx.download()
        assert r2["chi2_iter"] == r1["chi2_iter"] and r2["trials_iter"] == r1["trials_iter"]
        assert r2["pcg_iterations"] == r1["pcg_iterations"]
        for a, b in zip(s1, s2):
            assert np.array_equal(a, b)
        # damped solves at the solved state: g2o's initial damping (tau max diag H) and the LM's last
        b, d = ctx.gradient()
        out = []
        for lam in [rel * np.abs(d).max() for rel in lambdas_rel] + [r1["lambda_final"]]:
            x = ctx.damped_solve(lam, b, solver="pcg", max_iterations=4096)
            its, ok = ctx.last_step_info()
            assert ok and its > 0
            ax = ctx.hessian_product(x) + lam * x
            res = np.linalg.norm(b - ax)
            out.append((lam, its, res / np.linalg.norm(b)))
            assert res / np.linalg.norm(b) < 1e-11, out
            assert res / (np.linalg.norm(ax) + np.linalg.norm(b)) < 1e-12, out
        return r1, out


def test_c2_full_size_properties():
    r, solves = check_props(c2_problem(), 6, (1e-5,))
    print("C2", r["trials_iter"], solves)


def test_north_star_500k_properties():
    """The north-star size (500k correspondences x 2 views, 3,000,008 unknowns: bench.py's
    north_star_500k leg) on the tile chain — the largest tile plan: monotone accepted chi2, a
    bit-identical repeat, damped solves to a backward error < 1e-12."""
    p = sim.two_view_problem(500000, 1)
    assert p.n_unknowns == 3000008
    with capi.Context(0) as ctx:
        ctx.set_plan("auto")
        ctx.upload(p)
        assert ctx.plan_info()["tiles"] > 0
    r, solves = check_props(p, 3, (1e-5,))
    print("500k", r["trials_iter"], solves)


def test_c3_shape_full_size_properties():
    p = c3_problem()
    assert p.n_pairs == 28 and p.n_unknowns == 1200224
    r, solves = check_props(p, 3, (1e-5,))
    print("C3", r["trials_iter"], solves)


def test_c4_full_size_properties():
    """C4 (BASELINE configs[3]): 500k correspondences x 8 keyframes, all 28 pairs — 12,000,224
    unknowns, 84M ARAP edges (bench.py --workload c4's scene), the same properties over 2 LM
    iterations."""
    p = c4_problem()
    assert p.n_pairs == 28 and p.n_unknowns == 12000224
    r, solves = check_props(p, 2, (1e-5,))
    print("C4", r["trials_iter"], solves)


def c5_scene():
    """bench.py --workload c5's scene: Realcolon.yaml (KB8 d0..d3, rep 1, arap 0.1, DepthWeight 0.001 ->
    sigma_d 1e-6 m, Data/Realcolon.yaml:15-23,101,110), 20 keyframes x 200k, the 19 consecutive pairs"""
    am = sim.multi_view_arrays(n=200000, k=20, seed=1, kb8=sim.REALCOLON_KB8)
    host = capi.Context(-1)
    host.set_pair_window(1)
    p = host.build_graph(am, 1.0, 0.1, np.float32(1e-6))
    host.close()
    return p, am


def _apply(am, ids, pts, n):
    """the solved points (graph order, MapPoint id k * n + i) into the ArrayMap's keyframes"""
    ids = np.asarray(ids)
    k, i = ids // n, ids % n
    for kk in range(len(am.kfs)):
        sel = k == kk
        am.kfs[kk]["pos"][i[sel]] = pts[sel].astype(np.float32)


def test_c5_full_size_properties():
    """C5 (BASELINE configs[4]): Realcolon 20 keyframes x 200k, 19 consecutive pairs — 12,000,152
    unknowns (g2oBundleAdjustment.cc:640-962 over the sliding window).  The full-size properties over 3
    LM iterations, then the configuration's fp32-vs-fp64 sweep AT this size: the same 3 iterations with
    the ARAP Jacobians stored in fp32 for the product (deftri_set_jacobian_storage 1; b, the
    preconditioner, the vectors and every reduction stay fp64) take the same trials, and the reprojection
    RMSE of the solved map (calculatePixelsStandDev, Geometry.cc:370-498) is within the north-star
    1e-4 px of the fp64 run's."""
    p, am = c5_scene()
    assert p.n_pairs == 19 and p.n_unknowns == 12000152
    r64, solves = check_props(p, 3, (1e-5,))
    print("C5", r64["trials_iter"], solves)
    init = [kf["pos"].copy() for kf in am.kfs]
    rms, runs = {}, {}
    with capi.Context(0) as ctx:
        for fp32 in (0, 1):
            ctx.set_plan("auto")
            ctx.set_jacobian_storage(fp32)
            ctx.upload(p)
            info = ctx.plan_info()
            assert info["plan"] == "iterative" and bool(info["jacobian_fp32"]) == bool(fp32)
            r = ctx.solve_lm(3, analytic=False)
            pts, _, _ = ctx.download()
            assert r["pcg_fallbacks"] == 0
            for kk, kf in enumerate(am.kfs):
                kf["pos"][:] = init[kk]
            _apply(am, p.point_ids, pts, 200000)
            rms[fp32] = ctx.pixels_stand_dev(am)
            runs[fp32] = r
    assert runs[0]["chi2_iter"] == r64["chi2_iter"]           # the fp64 run is the properties' run
    assert runs[1]["trials_iter"] == runs[0]["trials_iter"]
    np.testing.assert_allclose(runs[1]["chi2_iter"], runs[0]["chi2_iter"], rtol=1e-6)
    for k in ("desv", "desvc1", "desvc2"):
        assert abs(rms[1][k] - rms[0][k]) < 1e-4, (k, rms)
    print("C5 fp32 vs fp64", {k: abs(rms[1][k] - rms[0][k]) for k in ("desv", "desvc1", "desvc2")})
