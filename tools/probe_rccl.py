"""Probe: can RCCL run two ranks on ONE GPU (the test box has one)?  Each rank runs the sharded
ARAP LM of a small problem over RCCL send/recv + all-reduce and prints its report.
  torchrun --nproc-per-node 2 tools/probe_rccl.py"""
import os
import sys
import pathlib

import torch
import torch.distributed as dist

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
import numpy as np  # noqa: E402

from deftri import capi, sim  # noqa: E402
from deftri import dist as ddist  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
m, _ = sim.simulate_two_view(n=3000, seed=2, scale_scene=True, compact=True)
host = capi.Context(-1)
p = host.build_graph(m, 1.0, 2e5, np.float32(0.003))
ctx = capi.Context(0)
try:
    ddist.init_rccl(ctx, rank, world)
except Exception as e:
    print(f"[rank {rank}] RCCL init failed: {e}", flush=True)
    sys.exit(0)
ctx.upload(p)
r = ctx.solve_lm(4)
print(f"[rank {rank}] RCCL sharded LM: it {r['iterations']} trials {r['trials_total']} chi2 {r['chi2_final']:.9e}", flush=True)
ctx2 = capi.Context(0)
if rank == 0:
    ctx2.upload(p)
    r2 = ctx2.solve_lm(4)
    print(f"[rank 0] single-GPU LM: it {r2['iterations']} trials {r2['trials_total']} chi2 {r2['chi2_final']:.9e}", flush=True)
dist.barrier()
