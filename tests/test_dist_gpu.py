"""Point-sharded ARAP LM on the device (deftri_dist_*): world_size 2 and 3 processes share the one
GPU of the test box (gloo host transport — RCCL needs one GPU per rank; the RCCL path of the same
transfers runs in bench.py --gpus N).  The sharded solve must follow the single-GPU LM trajectory
of the same problem: identical iteration / trial counts; chi2 per iteration and the gathered state
within rounding — the ranks sum their partial H, b and chi2 in a different order, and LM on this
ill-conditioned system (ARAP information arapW*T^2 ~ 1e15) grows a 1e-16 difference by a few
decades per iteration: analytic Jacobians rel 1e-8 over 6 iterations; g2o numeric Jacobians
(delta 1e-9 central differences amplify state differences ~1e7x) chi2 rel 1e-5, the tolerance of
the numeric-mode golden parity test."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_CORR, N_IT = 4000, 6


def _problem():
    from deftri import capi, sim
    m, _ = sim.simulate_two_view(n=N_CORR, seed=2, scale_scene=True, compact=True)
    host = capi.Context(-1)
    p = host.build_graph(m, 1.0, 2e5, np.float32(0.003))
    host.close()
    return p


def _worker(rank, world, port, q):
    import faulthandler
    import sys
    faulthandler.enable()
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deftri import capi
    from deftri import dist as ddist
    p = _problem()
    ctx = capi.Context(0)
    ctx.dist_set_transport(world, rank, ddist.torch_transport())
    ctx.set_plan("multifrontal")            # the sharded LDL^T (the iterative plan: test_gpu_sp.py)
    ctx.upload(p)
    res = {}
    for analytic in (True, False):
        ctx.reset_state()
        r = ctx.solve_lm(N_IT, analytic=analytic)
        print(f"[rank {rank}] analytic={analytic}: {r['iterations']} iterations, {r['trials_total']} trials, "
              f"chi2 {r['chi2_final']:.12e}", file=sys.stderr, flush=True)
        pts, sc, tg = ctx.download()
        owner = ctx.vertex_owner()
        P, S, T = ddist.gather_state(p, owner, rank, pts, sc, tg, lambda a: dist.all_reduce(torch.from_numpy(a)))
        res[analytic] = (r, P, S, T, owner)
    q.put((rank, res))
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_lm_matches_single_gpu(world):
    from deftri import capi
    cm = mp.get_context("spawn")
    q = cm.Queue()
    port = 29900 + 13 * world + os.getpid() % 500
    procs = [cm.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = {}
    for _ in procs:
        rank, *rest = q.get(timeout=240)
        out[rank] = rest
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p = _problem()
    ref = {}
    with capi.Context(0) as ctx:
        ctx.set_lm_lanes(1)
        ctx.set_plan("multifrontal")
        ctx.upload(p)
        for analytic in (True, False):
            ctx.reset_state()
            r = ctx.solve_lm(N_IT, analytic=analytic)
            ref[analytic] = (r, *ctx.download())
    for analytic, tol in ((True, 1e-8), (False, 1e-5)):
        rr, pts, sc, tg = ref[analytic]
        owner = out[0][0][analytic][4]
        assert set(np.unique(owner)) == set(range(world))
        for r in range(world):
            rep, P, S, T, _ = out[r][0][analytic]
            assert rep["nranks"] == world and rep["rank"] == r
            assert rep["iterations"] == rr["iterations"]
            assert rep["trials_total"] == rr["trials_total"]
            np.testing.assert_allclose(rep["chi2_iter"], rr["chi2_iter"], rtol=tol)
            assert rep["chi2_final"] == pytest.approx(rr["chi2_final"], rel=tol)
            assert rep["factor_flops_total"] == pytest.approx(rr["factor_flops"], rel=1e-12)
            assert np.abs(P - pts).max() <= tol * np.abs(pts).max()
            np.testing.assert_allclose(S, sc, rtol=tol)
            np.testing.assert_allclose(T, tg, rtol=tol, atol=tol * 1e-3)
