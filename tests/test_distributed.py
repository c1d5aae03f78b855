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
    dist.barrier()
    q.put((rank, t, it, tr))
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
    for rank, t, it, tr in out:
        assert t == pytest.approx(1.5) and it == 10 and tr == 25


def test_reduce_stats_single():
    import bench
    assert bench.reduce_stats(2.0, 3, 7, 1, "cpu") == (2.0, 3, 7)
