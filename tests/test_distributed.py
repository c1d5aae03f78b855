"""N>1 bench path on CPU: world_size-2 gloo ranks aggregate their replica timings the way
bench.py does on RCCL (max time over ranks, summed iterations)."""
import os

import pytest
import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    t, it, tr = bench.reduce_stats(0.5 + rank, 5, 12 + rank, world, "cpu")
    # the sharded ARAP line: both ranks ran the same 5 iterations of one problem
    t1, _, _ = bench.reduce_stats(0.020 + 0.005 * rank, 5, 9, world, "cpu")
    value, ms = bench.job_rate(t1, 5)
    weak, _ = bench.job_rate(t1, 5, world)          # weak scaling: world shares per iteration
    dist.barrier()
    q.put((rank, t, it, tr, value, ms, weak))
    dist.destroy_process_group()


def test_reduce_stats_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, t, it, tr, value, ms, weak in out:
        assert t == pytest.approx(1.5) and it == 10 and tr == 25
        # value = iterations of the one problem over the slowest rank's time (not a sum over ranks)
        assert value == pytest.approx(5 / 0.025) and ms == pytest.approx(5.0)
        # weak scaling: the problem has 2 C2-sized shares, so one of its iterations counts twice
        assert weak == pytest.approx(2 * 5 / 0.025)


def test_reduce_stats_single():
    import bench
    assert bench.reduce_stats(2.0, 3, 7, 1, "cpu") == (2.0, 3, 7)
