"""Bundle adjustment on the CPU: the oracle's BlockSolver_6_3 restatement
(oracle/ba_oracle.c) against independent formula checks, the map-level control flows of
deftri/ba.py driven by the oracle, and the point-sharded reduction algebra over world_size-2 gloo.

Parity of the device path with this oracle is in test_ba_gpu.py.  The reference's BA functions
have no tests or fixtures: parity unpinned, formula-checked here."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from ba_oracle_ctx import OracleBA
from deftri import ba
from oracle import oracle


def _se3_left(pose7, u):
    """T <- exp(u) * T with the oracle's SE3Quat::exp (VertexSE3Expmap::oplusImpl)."""
    import ctypes as C
    e = np.zeros(7)
    uu = np.ascontiguousarray(u, np.float64)
    oracle.lib().oracle_se3_exp(uu.ctypes.data_as(C.POINTER(C.c_double)), e.ctypes.data_as(C.POINTER(C.c_double)))
    qa, ta = e[:4], e[4:]
    qb, tb = pose7[:4], pose7[4:]
    from deftri.mapmodel import mat_from_quat
    Ra = mat_from_quat(qa)
    t = Ra @ tb + ta
    x1, y1, z1, w1 = qa
    x2, y2, z2, w2 = qb
    q = np.array([w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2, w1 * y2 + y1 * w2 + z1 * x2 - x1 * z2,
                  w1 * z2 + z1 * w2 + x1 * y2 - y1 * x2, w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2])
    if q[3] < 0:
        q = -q
    return np.concatenate([q / np.linalg.norm(q), t])


def _chi2_at(prob, poses, points):
    p2 = ba.BAProblem(poses, prob.pose_kb8, points, prob.edge_point, prob.edge_pose, prob.edge_obs, prob.edge_info,
                      pose_fixed=prob.pose_fixed, point_fixed=prob.point_fixed, edge_level=prob.edge_level,
                      edge_robust=prob.edge_robust)
    return oracle.ba_eval_system(p2, 1.0)["chi2"]


def test_oracle_gradient_matches_finite_differences():
    """b = -J^T rho' Omega e, so d(activeRobustChi2)/dx = -2 b (Huber's first derivative; g2o
    drops the second-order term only in H)."""
    p = ba.make_ba_problem(n=40, k=3, seed=3, outliers=0.1)
    s = oracle.ba_eval_system(p, 1.0)
    K = p.n_poses
    rng = np.random.default_rng(0)
    for _ in range(6):                      # point coordinates
        l, c = rng.integers(0, p.n_points), rng.integers(0, 3)
        h = 2e-4                            # fp32 projection: uv quantum ~3e-5 px
        pp, pm = p.points.copy(), p.points.copy()
        pp[l, c] += h; pm[l, c] -= h
        g = (_chi2_at(p, p.poses, pp) - _chi2_at(p, p.poses, pm)) / (2 * h)
        assert g == pytest.approx(-2 * s["b"][6 * K + 3 * l + c], rel=2e-3, abs=1e-2)
    # the fp32 projection leaves ~1e-7 relative noise on every chi2 term, so the difference quotient
    # of one component is only good to ~1e-5 of the largest gradient component
    gmax = np.abs(2 * s["b"][6:6 * K]).max()
    for k in (1, 2):                        # pose (rotation, translation), left-multiplied exp
        for c in range(6):
            h = 1e-4
            u = np.zeros(6); u[c] = h
            Pp, Pm = p.poses.copy(), p.poses.copy()
            Pp[k] = _se3_left(p.poses[k], u); Pm[k] = _se3_left(p.poses[k], -u)
            g = (_chi2_at(p, Pp, p.points) - _chi2_at(p, Pm, p.points)) / (2 * h)
            assert g == pytest.approx(-2 * s["b"][6 * k + c], rel=5e-3, abs=2e-5 * gmax)


def test_oracle_schur_step_solves_reduced_system():
    p = ba.make_ba_problem(n=60, k=4, seed=5)
    s = oracle.ba_eval_system(p, 10.0)
    assert s["ok"] and s["ns"] == 18          # KF 0 fixed
    S, rhs = s["S"], s["rhs"]
    assert np.abs(S - S.T).max() <= 1e-9 * np.abs(S).max()
    xp = np.concatenate([s["dx"][6 * k:6 * k + 6] for k in range(1, 4)])
    assert np.linalg.norm(S @ xp - rhs) <= 1e-10 * np.linalg.norm(S) * np.linalg.norm(xp)
    assert np.all(s["dx"][:6] == 0)           # fixed pose gets no step


def test_oracle_lm_descends_and_recovers_geometry():
    m, truth = ba.simulate_ba_map(n=150, k=4, seed=2)
    kfs = [m.keyframes[k] for k in m.kf_order()]
    prob, meta = ba.build_ba_graph(kfs)
    r = oracle.ba_solve(prob, 20)
    rep = r["report"]
    c = [rep["chi2_initial"]] + rep["chi2_iter"]
    assert all(b <= a for a, b in zip(c, c[1:]))
    assert rep["chi2_final"] < 0.2 * rep["chi2_initial"]
    # points approach the ground truth (the gauge is fixed by KF 0)
    err0 = np.linalg.norm(prob.points - truth["points"], axis=1).mean()
    err1 = np.linalg.norm(r["points"] - truth["points"], axis=1).mean()
    assert err1 < 0.5 * err0


def test_oracle_pose_only_and_levels():
    p = ba.make_ba_problem(n=80, k=2, seed=7, outliers=0.0)
    one = ba.BAProblem(p.poses[1:2], p.pose_kb8[1:2], p.points, p.edge_point[p.edge_pose == 1],
                       np.zeros(int((p.edge_pose == 1).sum()), np.int32), p.edge_obs[p.edge_pose == 1],
                       p.edge_info[p.edge_pose == 1], point_fixed=np.ones(p.n_points, np.uint8))
    r = oracle.ba_solve(one, 10)
    assert r["report"]["n_unknowns"] == 6
    assert r["report"]["chi2_final"] < r["report"]["chi2_initial"]
    # an edge on another level is inactive: its cached error stays untouched
    lv = np.zeros(one.n_edges, np.uint8); lv[0] = 1
    err0 = np.full((one.n_edges, 2), 7.0)
    r2 = oracle.ba_solve(one, 3, edge_level=lv, err=err0)
    assert np.all(r2["err"][0] == 7.0) and not np.any(r2["err"][1:] == 7.0)


@pytest.mark.parametrize("flow", ["bundle", "local", "pose_only"])
def test_map_flows_on_oracle(flow):
    m, truth = ba.simulate_ba_map(n=120, k=4, seed=4, outliers=0.05, visibility=0.9, min_common_obs=15)
    ctx = OracleBA()
    if flow == "bundle":
        rep = ba.bundleAdjustment(m, ctx=ctx)
        assert rep["chi2_final"] < rep["chi2_initial"]
    elif flow == "local":
        n_obs0 = sum(len(v) for v in m.kf_obs.values())
        rep = ba.localBundleAdjustment(m, 2, ctx=ctx)
        n_obs1 = sum(len(v) for v in m.kf_obs.values())
        assert rep["outliers_removed"] > 0 and n_obs0 - n_obs1 == rep["outliers_removed"]
        for kid, kf in m.keyframes.items():       # map tables stay consistent with the slots
            live = {mp.id for mp in kf.map_points if mp is not None}
            assert live == set(m.kf_obs[kid])
    else:
        kf = m.keyframes[3]
        n_before = sum(mp is not None for mp in kf.map_points)
        n_good = ba.poseOnlyOptimization(kf, ctx=ctx)
        assert 0 < n_good < n_before
        assert n_good == sum(mp is not None for mp in kf.map_points)


def _shard_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = ba.make_ba_problem(n=90, k=4, seed=9)
    sub, _, _ = p.shard(rank, world)
    lam = 5.0
    s = oracle.ba_eval_system(sub, lam)
    buf = torch.from_numpy(np.concatenate([s["S"].ravel(), s["rhs"], [s["chi2"]]]))
    dist.all_reduce(buf)
    q.put((rank, buf.numpy().copy()))
    dist.destroy_process_group()


def test_point_sharded_reduction_gloo_world2():
    """The multi-GPU decomposition: summing the per-shard reduced systems over ranks (what the
    device path all-reduces) gives the full system (the damping lambda I is added once per rank,
    hence (world - 1) lambda I extra)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 1000
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p = ba.make_ba_problem(n=90, k=4, seed=9)
    lam = 5.0
    full = oracle.ba_eval_system(p, lam)
    ns = full["ns"]
    for r in range(world):
        v = out[r]
        S = v[:ns * ns].reshape(ns, ns) - (world - 1) * lam * np.eye(ns)
        assert np.abs(S - full["S"]).max() <= 1e-9 * np.abs(full["S"]).max()
        assert np.abs(v[ns * ns:ns * ns + ns] - full["rhs"]).max() <= 1e-9 * np.abs(full["rhs"]).max()
        assert v[-1] == pytest.approx(full["chi2"], rel=1e-12)
