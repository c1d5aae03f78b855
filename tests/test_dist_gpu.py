"""Point-sharded ARAP LM on the device (deftri_dist_*): world_size 2 and 3 processes share the one
GPU of the test box (gloo host transport — RCCL needs one GPU per rank; the RCCL path of the same
transfers runs in bench.py --gpus N).  The sharded solve must follow the single-GPU LM trajectory
of the same problem (identical iteration / trial counts; chi2 per iteration and the gathered state
within rounding: the ranks sum their partial H, b and chi2 in a different order)."""
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
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deftri import capi
    from deftri import dist as ddist
    p = _problem()
    ctx = capi.Context(0)
    ctx.dist_set_transport(world, rank, ddist.torch_transport())
    ctx.upload(p)
    r = ctx.solve_lm(N_IT, analytic=False)
    pts, sc, tg = ctx.download()
    owner = ctx.vertex_owner()
    P, S, T = ddist.gather_state(p, owner, rank, pts, sc, tg, lambda a: dist.all_reduce(torch.from_numpy(a)))
    q.put((rank, r, P, S, T, owner))
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
    with capi.Context(0) as ctx:
        ctx.set_lm_lanes(1)
        ctx.upload(p)
        ref = ctx.solve_lm(N_IT, analytic=False)
        pts, sc, tg = ctx.download()
    owner = out[0][4]
    assert set(np.unique(owner)) == set(range(world))
    for r in range(world):
        rep, P, S, T, _ = out[r]
        assert rep["nranks"] == world and rep["rank"] == r
        assert rep["iterations"] == ref["iterations"]
        assert rep["trials_total"] == ref["trials_total"]
        np.testing.assert_allclose(rep["chi2_iter"], ref["chi2_iter"], rtol=1e-9)
        assert rep["chi2_final"] == pytest.approx(ref["chi2_final"], rel=1e-9)
        assert rep["factor_flops_total"] == pytest.approx(ref["factor_flops"], rel=1e-12)
        assert np.abs(P - pts).max() <= 1e-9 * np.abs(pts).max()
        np.testing.assert_allclose(S, sc, rtol=1e-9)
        np.testing.assert_allclose(T, tg, rtol=1e-9, atol=1e-12)
