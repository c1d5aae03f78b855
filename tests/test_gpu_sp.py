"""The iterative plan (deftri_set_plan ITERATIVE: point-sharded matrix-free PCG, csrc/spcg.h) on the
device, against the oracle (oracle/deftri_oracle.c: the reference LM with an exact SimplicialLDLT
step) and against the multifrontal plan.

Tolerances (the PCG stop test is 1e-12 on the recurrence residual):
  * gradient b and diag(H) rel 1e-13 vs the oracle's assembly
  * one damped solve: residual ||(H + lam I) x - b|| / ||b|| < 1e-11, rel 1e-8 vs the exact solve
  * LM trajectories (golden scenes, budget 4096): identical trial and iteration counts, chi2 per
    iteration rel 1e-5 (the golden scenes' weakly damped steps, as tests/test_gpu_pcg.py)
  * all-pairs 8-keyframe scene (BASELINE C3/C4 shape at 100 x 8; g2oBundleAdjustment.cc:640-953):
    identical trials, chi2 rel 1e-8 analytic / 1e-6 g2o numeric Jacobians
  * two-view 20k: iterative vs multifrontal plan, identical trials, chi2 rel 1e-8
  * sharded: 2 and 3 ranks sharing the GPU (gloo host transport; RCCL in bench.py) on a two-view and
    an all-pairs 8-keyframe scene: identical trials, chi2 rel 1e-8 analytic (1e-6 numeric), gathered
    state rel 1e-8 against the one-rank plan
  * fp32 Jacobian storage: identical trial counts on the golden-size all-pairs scene, RMSE within
    1e-4 px of the fp64 run
  * C5 shape (20 keyframes, Realcolon weights, 19 consecutive / all 190 pairs): identical trials,
    chi2 rel 1e-6, points rel 1e-6 vs the oracle"""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN
from deftri import capi, sim
from deftri.problem import Problem
from oracle import oracle

pytestmark = pytest.mark.gpu


def rel(a, b):
    return np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(np.asarray(b)), 1e-300)


def mv_problem(n=100, k=8, seed=1):
    m, _ = sim.simulate_multi_view(n=n, k=k, seed=seed)
    host = capi.Context(-1)
    p = host.build_graph(m, 1.0, 1e7, np.float32(0.3))
    host.close()
    return p


def tv_problem(n, seed=2):
    m, _ = sim.simulate_two_view(n=n, seed=seed, scale_scene=True, compact=True)
    host = capi.Context(-1)
    p = host.build_graph(m, 1.0, 2e5, np.float32(0.003))
    host.close()
    return p


def reprojection_rms(p, pts):
    """RMS over the reprojection edges of |obs - KB8(T_cw p)| (the oracle's fp32 projection), px."""
    import copy
    q = copy.copy(p)
    q.points = np.ascontiguousarray(pts, np.float64)
    e_rep, _, _ = oracle.edge_errors(q)
    return float(np.sqrt(np.mean(e_rep ** 2)))


@pytest.fixture
def it_ctx(gpu_ctx):
    gpu_ctx.set_plan("iterative")
    gpu_ctx.set_linear_solver("pcg", max_iterations=4096)
    yield gpu_ctx
    gpu_ctx.set_plan("multifrontal")
    gpu_ctx.set_linear_solver("pcg")
    gpu_ctx.set_jacobian_storage(0)


def test_iterative_gradient_and_solve_match_oracle(it_ctx, golden_cases):
    for p in [Problem.load(GOLDEN / g / "problem.npz") for g in golden_cases] + [mv_problem()]:
        it_ctx.upload(p)
        assert it_ctx.plan_info()["plan"] == "iterative"
        b_ref, H_ref, _ = oracle.linearize(p, analytic=True, dense=True)
        b, d = it_ctx.gradient()
        assert rel(b, b_ref) < 1e-13 and rel(d, np.diag(H_ref)) < 1e-13
        dmax = np.abs(np.diag(H_ref)).max()
        for lam_rel in (1e-2, 1.0):
            lam = lam_rel * dmax
            x = it_ctx.damped_solve(lam, b_ref, solver="pcg", max_iterations=4096)
            its, ok = it_ctx.last_step_info()
            assert ok and its > 0
            A = H_ref + lam * np.eye(len(b_ref))
            assert np.linalg.norm(A @ x - b_ref) / np.linalg.norm(b_ref) < 1e-11
            assert rel(x, oracle.damped_solve(p, lam, b_ref)) < 1e-8


def test_iterative_lm_matches_oracle_golden(it_ctx, golden_cases):
    for g in golden_cases:
        p = Problem.load(GOLDEN / g / "problem.npz")
        it_ctx.upload(p)
        r = it_ctx.solve_lm(10, analytic=True)
        ref = oracle.solve_lm(p, 10, analytic=True)["report"]
        assert r["iterations"] == ref["iterations"] and r["trials_total"] == ref["trials_total"]
        np.testing.assert_allclose(r["chi2_iter"], ref["chi2_iter"], rtol=1e-5)
        assert r["pcg_fallbacks"] == 0 and r["pcg_trials"] == r["trials_total"]


@pytest.mark.parametrize("analytic,tol", [(True, 1e-8), (False, 1e-6)])
def test_iterative_lm_all_pairs_matches_oracle(it_ctx, analytic, tol):
    """8 keyframes, all 28 pairs (the reference's pair loop), 100 correspondences per keyframe."""
    p = mv_problem()
    assert p.n_pairs == 28 and p.n_scales == 56
    it_ctx.upload(p)
    n_it = 6 if analytic else 4
    r = it_ctx.solve_lm(n_it, analytic=analytic)
    res = oracle.solve_lm(p, n_it, analytic=analytic)
    ref = res["report"]
    assert r["iterations"] == ref["iterations"] and r["trials_total"] == ref["trials_total"]
    np.testing.assert_allclose(r["chi2_iter"], ref["chi2_iter"], rtol=tol)
    assert r["pcg_trials"] == r["trials_total"]
    pts, sc, tg = it_ctx.download()
    assert np.abs(pts - res["points"]).max() <= 1e-6 * max(np.abs(res["points"]).max(), 1.0)
    np.testing.assert_allclose(sc, res["scales"], rtol=1e-6)


@pytest.mark.parametrize("n,window,n_it", [(60, 1, 4), (24, 0, 3)])
def test_iterative_lm_c5_shape_matches_oracle(it_ctx, n, window, n_it):
    """BASELINE C5's shape at test size: 20 keyframes, Realcolon weights (Data/Realcolon.yaml:15-23,
    101,110: KB8 with distortion, arap 0.1, DepthWeight 0.001 -> information 1e12), g2o numeric
    Jacobians; the 19 consecutive pairs of the timed C5 (pair window 1) and the reference's all 190
    pairs.  The oracle eliminates in the host analysis's order."""
    p = sim.multi_view_problem(n, 20, seed=3, kb8=sim.REALCOLON_KB8, rep_weight=1.0, arap_weight=0.1,
                               depth_sigma=np.float32(1e-6), pair_window=window)
    assert p.n_pairs == (19 if window == 1 else 190) and p.n_scales == 2 * p.n_pairs
    it_ctx.upload(p)
    r = it_ctx.solve_lm(n_it, analytic=False)
    with capi.Context(-1) as h:
        h.analyse(p)
        oracle.set_vertex_order(h.vertex_order())
    try:
        res = oracle.solve_lm(p, n_it, analytic=False)
    finally:
        oracle.set_vertex_order(None)
    ref = res["report"]
    assert r["iterations"] == ref["iterations"] and r["trials_total"] == ref["trials_total"]
    np.testing.assert_allclose(r["chi2_iter"], ref["chi2_iter"], rtol=1e-6)
    assert r["pcg_trials"] == r["trials_total"] and r["pcg_fallbacks"] == 0
    pts, sc, tg = it_ctx.download()
    assert np.abs(pts - res["points"]).max() <= 1e-6 * max(np.abs(res["points"]).max(), 1.0)


def test_iterative_matches_multifrontal_two_view(gpu_ctx):
    p = tv_problem(20000, seed=1)
    out = {}
    for plan in ("multifrontal", "iterative"):
        gpu_ctx.set_plan(plan)
        gpu_ctx.upload(p)
        gpu_ctx.set_linear_solver("pcg", max_iterations=4096)
        out[plan] = gpu_ctx.solve_lm(6, analytic=False)
        assert gpu_ctx.plan_info()["plan"] == plan
    gpu_ctx.set_plan("multifrontal")
    gpu_ctx.set_linear_solver("pcg")
    a, b = out["iterative"], out["multifrontal"]
    assert a["trials_total"] == b["trials_total"] and a["pcg_fallbacks"] == b["pcg_fallbacks"] == 0
    np.testing.assert_allclose(a["chi2_iter"], b["chi2_iter"], rtol=1e-8)


def test_iterative_repeatable_and_profiled(it_ctx):
    p = tv_problem(5000, seed=3)
    it_ctx.upload(p)
    r1 = it_ctx.solve_lm(3, analytic=False)
    pts1, _, _ = it_ctx.download()
    it_ctx.reset_state()
    r2 = it_ctx.solve_lm(3, analytic=False)
    pts2, _, _ = it_ctx.download()
    assert r1["chi2_iter"] == r2["chi2_iter"] and np.array_equal(pts1, pts2)   # fixed-order sums
    st = it_ctx.profile_trial(r1["lambda_final"])
    keys = ["sp_glin_rows", "sp_setup", "sp_phase1", "sp_phase2", "sp_heavy"]
    if it_ctx.plan_info()["cg_launches"] > 2:         # the merged chain updates in phase 2
        keys.append("sp_update")
    for k in keys:
        assert k in st and st[k]["launches"] > 0, k
    assert st["sp_phase1"]["bytes"] > 0 and st["sp_phase2"]["bytes"] > 0
    assert "update" not in st and "hchunk" not in st          # no factorization, no assembled H


def test_fp32_jacobian_storage(it_ctx):
    """C5's precision sweep on the timed path at test size: fp32-stored ARAP J in the product."""
    p = mv_problem(n=80, k=5, seed=4)
    res = {}
    for fp32 in (0, 1):
        it_ctx.set_jacobian_storage(fp32)
        it_ctx.upload(p)
        assert it_ctx.plan_info()["jacobian_fp32"] == fp32
        r = it_ctx.solve_lm(5, analytic=False)
        res[fp32] = (r, it_ctx.download()[0])
    assert res[0][0]["trials_total"] == res[1][0]["trials_total"]
    np.testing.assert_allclose(res[1][0]["chi2_iter"], res[0][0]["chi2_iter"], rtol=1e-3)
    # reprojection RMS (px) of the final points, fp32 vs fp64 storage
    e = [reprojection_rms(p, pts) for pts in (res[0][1], res[1][1])]
    assert abs(e[0] - e[1]) < 1e-4, e


# ---- sharded: ranks sharing the GPU over the gloo host transport ----------------------------------
def _problem(kind):
    return tv_problem(4000, seed=2) if kind == "tv" else mv_problem(n=120, k=8, seed=2)


def _worker(rank, world, port, kind, q):
    import faulthandler
    import sys
    faulthandler.enable()
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deftri import capi as c
    from deftri import dist as ddist
    p = _problem(kind)
    ctx = c.Context(0)
    ctx.dist_set_transport(world, rank, ddist.torch_transport())
    ctx.set_linear_solver("pcg", max_iterations=4096)
    ctx.upload(p)
    info = ctx.plan_info()
    res = {}
    for analytic in (True, False):
        ctx.reset_state()
        r = ctx.solve_lm(4, analytic=analytic)
        print(f"[rank {rank}] {kind} analytic={analytic}: {r['trials_total']} trials chi2 {r['chi2_final']:.12e}",
              file=sys.stderr, flush=True)
        pts, sc, tg = ctx.download()
        owner = ctx.vertex_owner()
        P, S, T = ddist.gather_state(p, owner, rank, pts, sc, tg, lambda a: dist.all_reduce(torch.from_numpy(a)))
        res[analytic] = (r, P, S, T)
    q.put((rank, info, res))
    ctx.close()
    dist.destroy_process_group()


def oracle_lm(p, n_it, analytic):
    """The oracle's LM (exact SimplicialLDLT steps) eliminating in the host analysis's order."""
    with capi.Context(-1) as h:
        h.analyse(p)
        oracle.set_vertex_order(h.vertex_order())
    try:
        return oracle.solve_lm(p, n_it, analytic=analytic)
    finally:
        oracle.set_vertex_order(None)


@pytest.mark.parametrize("kind", ["tv", "mv"])
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_iterative_matches_oracle(kind, world):
    """2 and 3 ranks sharing the GPU (gloo host transport) against the oracle's LM on the same
    problem: a two-view scene and the 8-keyframe all-pairs scene (g2oBundleAdjustment.cc:640-953)."""
    cm = mp.get_context("spawn")
    q = cm.Queue()
    port = 28900 + 31 * world + (7 if kind == "mv" else 0) + os.getpid() % 300
    procs = [cm.Process(target=_worker, args=(r, world, port, kind, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = {}
    for _ in procs:
        rank, info, res = q.get(timeout=300)
        out[rank] = (info, res)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p = _problem(kind)
    assert sum(out[r][0]["own_rows"] for r in range(world)) == p.n_points
    for r in range(world):
        info = out[r][0]
        assert info["plan"] == "iterative" and info["nranks"] == world and info["halo_rows"] > 0
        assert info["sharded"] == 1 and info["cg_launches"] == 3 and info["cg_collectives"] == 1
        assert (info["tiles"] > 0) == (kind == "tv")   # one pair: the sharded tile chain (spcg_tile.cpp)
    # the sharded chain (single-reduction CG, sums split over the ranks) against exact steps: the
    # step differences are ~kappa * 1e-12 and the LM iterations amplify them
    for analytic, tol in ((True, 1e-8), (False, 1e-6)):
        res = oracle_lm(p, 4, analytic)
        ref = res["report"]
        for r in range(world):
            rep, P, S, T = out[r][1][analytic]
            assert rep["nranks"] == world and rep["rank"] == r
            assert rep["iterations"] == ref["iterations"] and rep["trials_total"] == ref["trials_total"]
            assert rep["trials_iter"] == ref["trials_iter"]
            np.testing.assert_allclose(rep["chi2_iter"], ref["chi2_iter"], rtol=tol)
            assert np.abs(P - res["points"]).max() <= 10 * tol * np.abs(res["points"]).max()
            np.testing.assert_allclose(S, res["scales"], rtol=10 * tol)


def test_iterative_plan_reuse_matches_fresh_upload():
    """An upload with the uploaded problem's structure and ordering coordinates (NLopt's evaluations:
    the same graph under other weights) keeps the iterative plan and copies only the values; the LM
    result is bit-identical to a fresh context's."""
    m, _ = sim.simulate_two_view(n=20000, seed=4, scale_scene=True, compact=True)
    host = capi.Context(-1)
    p1 = host.build_graph(m, 1.0, 2e5, np.float32(0.003))
    p2 = host.build_graph(m, 2.0, 5e4, np.float32(0.01))
    host.close()
    a, b = capi.Context(0), capi.Context(0)
    try:
        for c in (a, b):
            c.set_plan("iterative")
        a.upload(p1)
        a.solve_lm(3)
        a.upload(p2)
        ra = a.solve_lm(5)
        b.upload(p2)
        rb = b.solve_lm(5)
        assert ra["plan_reuses"] == 1 and rb["plan_reuses"] == 0
        assert ra["trials_iter"] == rb["trials_iter"]
        assert ra["chi2_iter"] == rb["chi2_iter"]
        for x, y in zip(a.download(), b.download()):
            assert np.array_equal(x, y)
    finally:
        a.close()
        b.close()


def _fusion_worker(env, q):
    # the two-phase chains unless the run asks for the tile chain (DEFTRI_SP_TILE)
    env = dict(env) if "DEFTRI_SP_TILE" in env else {"DEFTRI_SP_NO_TILE": "1", **env}
    os.environ.update(env)                          # read once, at the first upload of this process
    from deftri import capi as c
    p = tv_problem(20000, seed=6)
    with c.Context(0) as ctx:
        ctx.set_plan("iterative")
        ctx.upload(p)
        info = ctx.plan_info()
        r = ctx.solve_lm(5)
        q.put((info["cg_launches"], r["chi2_iter"], r["trials_iter"], r["pcg_iterations"],
               [a.tobytes() for a in ctx.download()]))


def _fusion_runs(envs, worker=None):
    cm = mp.get_context("spawn")
    out = []
    for env in envs:
        q = cm.Queue()
        pr = cm.Process(target=worker or _fusion_worker, args=(env, q))
        pr.start()
        out.append(q.get(timeout=300))
        pr.join(timeout=60)
        assert pr.exitcode == 0
    return out


def test_fused_cg_chain_matches_unfused():
    """One rank: the dots in the update's last workgroup and the heavy finish in the product's last
    workgroup (3 launches per CG iteration, DEFTRI_SP_NO_MERGE=1) form the same sums in the same order
    as the separate k_sp_dots / k_sp_heavy launches (DEFTRI_SP_NO_FUSE=1): bit-identical LM runs."""
    (l0, c0, t0, i0, s0), (l1, c1, t1, i1, s1) = _fusion_runs(
        [{"DEFTRI_SP_NO_MERGE": "1"}, {"DEFTRI_SP_NO_FUSE": "1"}])
    assert l0 == 3 and l1 == 5
    assert c0 == c1 and t0 == t1 and i0 == i1
    assert s0 == s1


def test_merged_cg_chain_matches_three_launch_chain():
    """One rank, merged chain (2 launches per CG iteration: p.Ap and alpha in phase 1, the update and
    the next (r.z, r.r) in phase 2) vs the three-launch chain (alpha from p.q after phase 2): the same
    CG in exact arithmetic, with p.Ap summed as sum_e W_e (J_e p)^2 + row / heavy terms instead of
    sum_v p_v q_v, so the steps differ at rounding level.  Tolerances: identical trials and CG
    iteration counts, chi2 rel 1e-8, states within 1e-7 of their largest magnitude."""
    (l0, c0, t0, i0, s0), (l1, c1, t1, i1, s1) = _fusion_runs([{}, {"DEFTRI_SP_NO_MERGE": "1"}])
    assert l0 == 2 and l1 == 3
    assert t0 == t1 and i0 == i1
    np.testing.assert_allclose(c0, c1, rtol=1e-8)
    for a, b in zip(s0, s1):
        x, y = np.frombuffer(a), np.frombuffer(b)
        assert np.max(np.abs(x - y)) <= 1e-7 * max(np.max(np.abs(y)), 1.0)


def test_phase2_step_size_bit_identical():
    """Phase 2's slot loop in chunks of 4, 6 or 8 slots (DEFTRI_SP_P2_STEP): the same
    adds in the same slot order (a clamped last step adds exact zeros) — bit-identical LM runs; the
    same for k_sp_glin_rows' step (DEFTRI_SP_GLIN_STEP)."""
    runs = _fusion_runs([{"DEFTRI_SP_P2_STEP": "4"}, {"DEFTRI_SP_P2_STEP": "6"}, {"DEFTRI_SP_P2_STEP": "8"},
                         {"DEFTRI_SP_GLIN_STEP": "4"}, {"DEFTRI_SP_GLIN_STEP": "6"}, {"DEFTRI_SP_GLIN_STEP": "8"}])
    for l, c, t, i, s in runs[1:]:
        assert l == runs[0][0] == 2
        assert c == runs[0][1] and t == runs[0][2] and i == runs[0][3]
        assert s == runs[0][4]


@pytest.mark.parametrize("rs", ["1", "4"])
def test_phase2_row_split_matches(rs):
    """Phase 2 with each row's slot list split over rs waves (DEFTRI_SP_ROW_SPLIT; default 2): q_v is
    summed as (part 0 + part 1 ...) instead of in one run, so the steps differ at rounding level.
    Tolerances as for the merged vs three-launch chains: identical trials and CG iteration counts,
    chi2 rel 1e-8, states within 1e-7 of their largest magnitude."""
    (l0, c0, t0, i0, s0), (l1, c1, t1, i1, s1) = _fusion_runs([{}, {"DEFTRI_SP_ROW_SPLIT": rs}])
    assert l0 == l1 == 2
    assert t0 == t1 and i0 == i1
    np.testing.assert_allclose(c0, c1, rtol=1e-8)
    for a, b in zip(s0, s1):
        x, y = np.frombuffer(a), np.frombuffer(b)
        assert np.max(np.abs(x - y)) <= 1e-7 * max(np.max(np.abs(y)), 1.0)


def _arap_j_worker(env, negz, q):
    os.environ.update(env)
    from deftri import capi as c
    p = tv_problem(20000, seed=6)
    if negz:                                        # -0.0 coordinates: the full-evaluation path
        pts = p.points.copy()
        for i in p.arap_pts[:50, 0]:
            pts[i, 1] = -0.0
        p.points = pts
    with c.Context(0) as ctx:
        ctx.set_plan("iterative")
        ctx.upload(p)
        r = ctx.solve_lm(4, analytic=False)
        q.put((r["chi2_iter"], r["trials_iter"], r["pcg_iterations"], [a.tobytes() for a in ctx.download()]))


@pytest.mark.parametrize("negz", [False, True])
def test_numeric_arap_jacobian_piece_reuse_bit_identical(negz):
    """k_lin_arap<2> (g2o's numeric ARAP Jacobian with the pieces a perturbed evaluation shares with
    the unperturbed one reused: no division for a T_g perturbation, 2 of 6 for a v2 one) against
    k_lin_arap<3> (every one of the 36 evaluations in full, DEFTRI_ARAP_J_FULL=1): the same bits, so
    bit-identical LM runs; with -0.0 coordinates (the edges that take the full path) too."""
    cm = mp.get_context("spawn")
    out = []
    for env in ({}, {"DEFTRI_ARAP_J_FULL": "1"}):
        qq = cm.Queue()
        pr = cm.Process(target=_arap_j_worker, args=(env, negz, qq))
        pr.start()
        out.append(qq.get(timeout=300))
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert out[0] == out[1]


@pytest.mark.parametrize("merge", ["1", ""])
def test_iterative_budget_exhausted_trials_rejected(merge):
    """A trial whose PCG exhausts its budget is rejected like a failed g2o linear solve (the
    iterative plan has no factorization behind it; g2o's solve() then returns false, the trial
    counts as rho < 0): lambda *= nu, nu *= 2.  With a budget no step meets at the first dampings
    (2 CG iterations to 1e-12) and max_trials = 3, the first LM iteration rejects its 3 trials and
    g2o's Terminate fires (qmax == maxTrials): chi2 and the state unchanged, lambda = tau max diag H *
    2 * 4 * 8 — the trajectory pinned without an oracle run.  (At far larger dampings H + lambda I is
    nearly its own block diagonal and 2 iterations do meet 1e-12.)  Both chains (merged; three-launch)."""
    import subprocess, sys, json as _json
    code = f"""
import os, sys, json
os.environ['DEFTRI_SP_{'MERGE' if merge else 'NO_MERGE'}'] = '1'
sys.path.insert(0, {str(capi.__file__.rsplit('/deftri/', 1)[0])!r})
sys.path.insert(0, {str(__file__.rsplit('/', 1)[0])!r})
import numpy as np
from test_gpu_sp import tv_problem
from deftri import capi
p = tv_problem(20000, seed=6)
with capi.Context(0) as ctx:
    ctx.set_plan('iterative')
    ctx.set_linear_solver('pcg', 1e-12, 2)
    ctx.upload(p)
    s0 = [a.tobytes() for a in ctx.download()]
    g, d = ctx.gradient()
    r = ctx.solve_lm(5, analytic=True, max_trials=3)
    s1 = [a.tobytes() for a in ctx.download()]
print(json.dumps(dict(r=dict((k, r[k]) for k in ('trials_total', 'trials_rejected', 'pcg_fallbacks', 'pcg_trials',
      'iterations', 'status', 'chi2_initial', 'chi2_final', 'lambda_final', 'cg_launches') if k in r),
      same=s0 == s1, maxdiag=float(np.abs(d).max()))))
"""
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-2000:]
    res = _json.loads(out.stdout.strip().splitlines()[-1])
    r = res["r"]
    assert r["trials_total"] == 3 and r["trials_rejected"] == 3, r
    assert r["pcg_fallbacks"] == 3 and r["pcg_trials"] == 0
    assert r["iterations"] == 1 and r["status"] == 1            # DEFTRI_STATUS_TERMINATE
    assert r["chi2_final"] == r["chi2_initial"]
    assert res["same"]
    assert r["lambda_final"] == pytest.approx(1e-5 * res["maxdiag"] * 2.0 ** 6, rel=1e-12)


def test_merged_chain_breakdown_then_solve():
    """A solve that breaks down inside the merged chain (a NaN in the right-hand side: p.Ap is NaN, so
    phase 2's workgroup 0 finds the breakdown while the other workgroups are running) fails loudly and
    leaves the plan as it found it: every workgroup still draws its ticket, and the next solve on the
    same plan — and an LM run after it — equal a fresh context's bit for bit."""
    p = tv_problem(20000, seed=7)                   # 60k unknowns: the merged chain
    a, b = capi.Context(0), capi.Context(0)
    try:
        for c in (a, b):
            c.set_plan("iterative")
            c.upload(p)
        assert a.plan_info()["cg_launches"] in (1, 2)         # the tile chain (one rank, one pair)
        g, d = a.gradient()
        lam = 1e-3 * np.abs(d).max()
        bad = g.copy()
        bad[len(bad) // 2] = np.nan
        with pytest.raises(capi.DeftriError):
            a.damped_solve(lam, bad, solver="pcg", max_iterations=4096)
        its_bad, ok_bad = a.last_step_info()
        assert not ok_bad
        xa = a.damped_solve(lam, g, solver="pcg", max_iterations=4096)
        ia = a.last_step_info()
        xb = b.damped_solve(lam, g, solver="pcg", max_iterations=4096)
        ib = b.last_step_info()
        assert ia == ib and ia[1] and np.array_equal(xa, xb)
        ra, rb = a.solve_lm(3), b.solve_lm(3)
        assert ra["chi2_iter"] == rb["chi2_iter"] and ra["trials_iter"] == rb["trials_iter"]
    finally:
        a.close()
        b.close()


def test_rccl_one_rank_sharded_chain():
    """The production transport on the one-GPU box: an RCCL communicator of one rank puts the
    iterative plan on the sharded control flow — the single-reduction CG chain (3 launches and one
    ncclAllReduce per CG iteration), chi2 / H / trial scalars through ncclAllReduce on the solver
    stream — against the oracle's LM."""
    p = tv_problem(4000, seed=2)
    c = capi.Context(0)
    try:
        c.dist_init_rccl(1, 0, capi.rccl_unique_id())
        c.set_plan("iterative")
        c.set_linear_solver("pcg", max_iterations=4096)
        c.upload(p)
        info = c.plan_info()
        assert info["plan"] == "iterative" and info["sharded"] == 1
        assert info["cg_launches"] == 3 and info["cg_collectives"] == 1
        for analytic, tol in ((True, 1e-8), (False, 1e-6)):
            c.reset_state()
            r = c.solve_lm(4, analytic=analytic)
            pts, sc, tg = c.download()
            res = oracle_lm(p, 4, analytic)
            ref = res["report"]
            assert r["iterations"] == ref["iterations"] and r["trials_iter"] == ref["trials_iter"]
            np.testing.assert_allclose(r["chi2_iter"], ref["chi2_iter"], rtol=tol)
            assert r["pcg_fallbacks"] == 0
            assert np.abs(pts - res["points"]).max() <= 10 * tol * np.abs(res["points"]).max()
    finally:
        c.close()


def test_device_lm_matches_host_lm():
    """The device-driven LM (k_lm_decide: rho, accept / reject, lambda / nu, g2o's Terminate test in
    HBM; the host queues trial slots without reading each outcome) against the host loop
    (the default): the same decisions from the same sums — bit-identical LM runs."""
    (l0, c0, t0, i0, s0), (l1, c1, t1, i1, s1) = _fusion_runs([{"DEFTRI_DEVICE_LM": "1"}, {}])
    assert l0 == l1 == 2
    assert c0 == c1 and t0 == t1 and i0 == i1
    assert s0 == s1


def _timeout_worker(env, q):
    os.environ.update(env)                          # read once, at the first upload of this process
    from deftri import capi as c
    p = tv_problem(20000, seed=6)                   # 60k unknowns: the merged chain
    with c.Context(0) as ctx:
        ctx.set_plan("iterative")
        ctx.upload(p)
        code, state_after_error = None, None
        if "DEFTRI_SP_INJECT_TIMEOUT_IT" in env:
            try:
                ctx.solve_lm(5)
            except c.DeftriError as e:
                code = e.code
            state_after_error = [a.tobytes() for a in ctx.download()]
        r = ctx.solve_lm(5)
        q.put((code, state_after_error, ctx.plan_info()["cg_launches"], r["chi2_iter"], r["trials_iter"],
               r["pcg_iterations"], [a.tobytes() for a in ctx.download()],
               [np.ascontiguousarray(x).tobytes() for x in (p.points, p.scales)]))


@pytest.mark.parametrize("lm", ["host", "device"])
def test_alpha_hand_off_timeout_is_an_error(lm):
    """A merged-chain alpha hand-off that times out (forced at CG iteration 1 by
    DEFTRI_SP_INJECT_TIMEOUT_IT) fails the call with DEFTRI_E_HIP on BOTH LM paths — never a rejected
    trial (the ADVICE r4 finding: the device-driven LM's k_lm_decide used to count it as a failed solve
    and raise lambda).  The state the call started from is restored, the context switches to the
    separate alpha launch, and the retried call equals a clean run bit for bit."""
    extra = {"DEFTRI_DEVICE_LM": "1"} if lm == "device" else {}
    extra["DEFTRI_SP_NO_TILE"] = "1"               # the merged two-phase chain (tile mode has no hand-off)
    faulted, clean = _fusion_runs_full([{"DEFTRI_SP_INJECT_TIMEOUT_IT": "1", **extra}, extra])
    code, state, launches, chi, trials, its, final, init = faulted
    assert code == -2                                # DEFTRI_E_HIP
    assert state[0] == init[0] and state[1] == init[1]   # points, scales as uploaded
    assert launches == 3                             # now the separate alpha launch
    assert chi == clean[3] and trials == clean[4] and its == clean[5]
    assert final == clean[6]


def _fusion_runs_full(envs):
    cm = mp.get_context("spawn")
    out = []
    for env in envs:
        q = cm.Queue()
        pr = cm.Process(target=_timeout_worker, args=(env, q))
        pr.start()
        out.append(q.get(timeout=300))
        pr.join(timeout=60)
        assert pr.exitcode == 0
    return out


def test_tile_chain_matches_two_phase_chain():
    """Tile mode (csrc/spcg_tile.cpp; one rank, one pair — the timed C2 chain): the product and the
    update as two launches against the two-phase merged chain (q summed in another order): identical
    trials and CG iteration counts, chi2 rel 1e-9.  The device-driven LM on the tile chain takes the
    host loop's decisions: bit for bit."""
    runs = _fusion_runs([{"DEFTRI_SP_TILE": "1"}, {}, {"DEFTRI_SP_TILE": "1", "DEFTRI_DEVICE_LM": "1"}])
    (l0, c0, t0, i0, s0), (l2, c2, t2, i2, s2), (l3, c3, t3, i3, s3) = runs
    assert l0 == 2 and l2 == 2
    assert t0 == t2 and i0 == i2
    np.testing.assert_allclose(c0, c2, rtol=1e-9)
    assert c3 == c0 and t3 == t0 and i3 == i0 and s3 == s0


def _ovl_worker(rank, world, port, env, q):
    os.environ.update(env)
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deftri import capi as c
    from deftri import dist as ddist
    p = _problem("mv")
    ctx = c.Context(0)
    ctx.dist_set_transport(world, rank, ddist.torch_transport())
    ctx.set_linear_solver("pcg", max_iterations=4096)
    ctx.upload(p)
    info = ctx.plan_info()
    r = ctx.solve_lm(4, analytic=False)
    pts, sc, tg = ctx.download()
    q.put((rank, info, r["chi2_iter"], r["trials_iter"], r["pcg_iterations"], pts.tobytes(), sc.tobytes(), tg.tobytes()))
    ctx.close()
    dist.destroy_process_group()


def test_sharded_halo_overlap_matches_serialized():
    """The sharded chain's halo exchange beside the interior product (phase-1 workgroups that read no
    halo row run while the boundary rows' (z, p) travel on a second stream; the others wait for them;
    SURVEY §8(e)) against the serialized order (DEFTRI_SP_NO_OVERLAP=1): the same workgroups compute
    the same sums, only their launch order differs — bit-identical LM runs at 2 ranks on the
    8-keyframe all-pairs scene, and plan_info reports the overlap."""
    cm = mp.get_context("spawn")
    runs = []
    for k, env in enumerate(({}, {"DEFTRI_SP_NO_OVERLAP": "1"})):
        q = cm.Queue()
        port = 29420 + 17 * k + os.getpid() % 300
        procs = [cm.Process(target=_ovl_worker, args=(r, 2, port, env, q)) for r in range(2)]
        for pr in procs:
            pr.start()
        out = {}
        for _ in procs:
            res = q.get(timeout=300)
            out[res[0]] = res[1:]
        for pr in procs:
            pr.join(timeout=60)
            assert pr.exitcode == 0
        runs.append(out)
    for r in range(2):
        assert runs[0][r][0]["halo_overlap"] == 1 and runs[1][r][0]["halo_overlap"] == 0
        assert runs[0][r][1:] == runs[1][r][1:]


_EXIT_CHILD = r"""
import sys
sys.path.insert(0, {pkg!r})
sys.path.insert(0, {tests!r})
import numpy as np
from test_gpu_sp import tv_problem
from deftri import ba, capi
keep = []
capi.Context.__del__ = lambda self: None          # the caller never destroys its contexts
capi.BAContext.__del__ = lambda self: None
p = tv_problem(20000, seed=6)
ctx = capi.Context(0)                              # the tile chain (one pair, >= 50k unknowns)
ctx.set_plan("iterative")
ctx.upload(p)
assert ctx.plan_info()["tiles"] > 0
ctx.solve_lm(3)
keep.append(ctx)
sd = capi.Context(0)                               # the sharded chain on a one-rank RCCL communicator
sd.dist_init_rccl(1, 0, capi.rccl_unique_id())
sd.set_plan("iterative")
sd.upload(p)
assert sd.plan_info()["sharded"] == 1
sd.solve_lm(3)
keep.append(sd)
m, _ = ba.simulate_ba_map(n=200, k=3, seed=2)      # a BA context
bc = capi.BAContext(0)
prob, _ = ba.build_ba_graph([m.keyframes[k] for k in m.kf_order()])
bc.upload(prob)
bc.solve_lm(5)
keep.append(bc)
print("done", flush=True)
sys.exit(0)
"""


def test_process_exit_with_live_contexts_is_clean():
    """Round 5 saw one SIGSEGV inside exit() after a clean run (the fused tile chain's cooperative
    launch under rocprofv3; that variant is removed).  A process that exits with its contexts still
    live — the tile chain, the sharded chain on an RCCL communicator and a BA context, none destroyed
    by the caller — must exit 0: the library releases them in an exit handler that runs before the HIP
    runtime's own teardown (csrc/exit_guard.h)."""
    import subprocess
    import sys
    code = _EXIT_CHILD.format(pkg=str(capi.__file__.rsplit("/deftri/", 1)[0]), tests=str(__file__.rsplit("/", 1)[0]))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "done" in r.stdout, (r.returncode, r.stderr[-3000:])


def _multi_tile_worker(env, q):
    # the tile chain below kSpMergeMinDof unknowns: DEFTRI_SP_MERGE=1 (read once per process)
    os.environ.update(env)
    from deftri import capi as c
    kind, n_it, analytic = env["_KIND"], int(env["_NIT"]), env["_ANALYTIC"] == "1"
    if kind == "mv":
        p = mv_problem()
    else:
        n, w = (60, 1) if kind == "c5w" else (24, 0)
        p = sim.multi_view_problem(n, 20, seed=3, kb8=sim.REALCOLON_KB8, rep_weight=1.0, arap_weight=0.1,
                                   depth_sigma=np.float32(1e-6), pair_window=w)
    with c.Context(0) as ctx:
        ctx.set_plan("iterative")
        ctx.set_linear_solver("pcg", max_iterations=4096)
        ctx.upload(p)
        info = ctx.plan_info()
        r = ctx.solve_lm(n_it, analytic=analytic)
        pts, sc, tg = ctx.download()
        q.put((info["tiles"], info["cg_launches"], r["iterations"], r["trials_iter"], r["chi2_iter"],
               r["pcg_trials"], r["trials_total"], r["pcg_fallbacks"], pts.tobytes(), sc.tobytes()))


@pytest.mark.parametrize("kind,n_it,analytic,tol", [("mv", 6, True, 1e-8), ("mv", 4, False, 1e-6),
                                                     ("c5w", 4, False, 1e-6), ("c5all", 3, False, 1e-6)])
def test_multi_pair_tile_chain_matches_oracle(kind, n_it, analytic, tol):
    """Tile mode over several keyframe pairs (csrc/spcg_tile.cpp build_tiles_multi; the chain C3-C5
    time): 8 keyframes with all 28 pairs (the reference's pair loop, g2oBundleAdjustment.cc:640-645),
    and BASELINE C5's shape — 20 keyframes under the Realcolon weights with the 19 consecutive pairs
    and with all 190 — against the oracle's LM: the same iterations and trials, chi2 per iteration and
    the solved points to the all-pairs test's tolerances; every trial solved by PCG on the tile chain
    (tiles > 0, two launches per CG iteration)."""
    env = {"DEFTRI_SP_MERGE": "1", "_KIND": kind, "_NIT": str(n_it), "_ANALYTIC": "1" if analytic else "0"}
    (tiles, launches, its, trials, chi2, pcg_trials, trials_total, fallbacks, pts, sc), = _fusion_runs([env], _multi_tile_worker)
    assert tiles > 0 and launches == 2
    if kind == "mv":
        p = mv_problem()
        res = oracle.solve_lm(p, n_it, analytic=analytic)
    else:
        n, w = (60, 1) if kind == "c5w" else (24, 0)
        p = sim.multi_view_problem(n, 20, seed=3, kb8=sim.REALCOLON_KB8, rep_weight=1.0, arap_weight=0.1,
                                   depth_sigma=np.float32(1e-6), pair_window=w)
        with capi.Context(-1) as h:
            h.analyse(p)
            oracle.set_vertex_order(h.vertex_order())
        try:
            res = oracle.solve_lm(p, n_it, analytic=analytic)
        finally:
            oracle.set_vertex_order(None)
    ref = res["report"]
    assert its == ref["iterations"] and trials_total == ref["trials_total"]
    np.testing.assert_allclose(chi2, ref["chi2_iter"], rtol=tol)
    assert pcg_trials == trials_total and fallbacks == 0
    pts = np.frombuffer(pts).reshape(-1, 3)
    assert np.abs(pts - res["points"]).max() <= 1e-6 * max(np.abs(res["points"]).max(), 1.0)
    np.testing.assert_allclose(np.frombuffer(sc), res["scales"], rtol=1e-6)
