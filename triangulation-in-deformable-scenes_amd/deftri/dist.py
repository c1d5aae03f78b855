"""Point-sharded ARAP solve across ranks (one process per GPU): the host pieces around the C-ABI's
deftri_dist_* entry points.

  * `torch_transport()` — the host-memory transport of deftri_dist_set_transport over an
    initialised torch.distributed process group (gloo: CPU tests, or several ranks sharing one
    GPU; the production path is RCCL, `Context.dist_init_rccl`).
  * `init_rccl(ctx, rank, world)` — one RCCL communicator per context; the 128-byte id travels from
    rank 0 through the process group.
  * `gather_state(...)` — every rank's authoritative part (deftri_dist_vertex_owner) of the solved
    state, summed over the ranks, so every rank ends with the whole solution (download side of
    arapOptimization's write-back, g2oBundleAdjustment.cc:967-1007).
"""
import numpy as np


def torch_transport():
    import torch
    import torch.distributed as dist

    def xfer(op, peer, arr):
        t = torch.from_numpy(arr)               # shares the staging buffer
        if op == 0:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elif op == 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elif op == 2:
            dist.send(t, peer)
        elif op == 3:
            dist.recv(t, peer)
        else:
            return -1
        return 0
    return xfer


def init_rccl(ctx, rank, world):
    import torch.distributed as dist
    from . import capi
    uid = [capi.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    ctx.dist_init_rccl(world, rank, uid[0])


def owner_masks(prob, owner, rank):
    """Per-entry masks of the state arrays (tg [Q,7], scales [S], points [P,3]) this rank is
    authoritative for; owner is deftri_dist_vertex_owner (vertex order [T_g][scales][points])."""
    Q, S = prob.n_pairs, prob.n_scales
    return owner[:Q] == rank, owner[Q:Q + S] == rank, owner[Q + S:] == rank


def gather_state(prob, owner, rank, pts, sc, tg, allreduce):
    """Combine the ranks' downloads: each rank contributes its authoritative vertices, `allreduce`
    sums a float64 numpy array in place over the ranks."""
    mt, ms, mp = owner_masks(prob, owner, rank)
    buf = np.concatenate([(tg.reshape(-1, 7) * mt[:, None]).ravel(), sc * ms, (pts.reshape(-1, 3) * mp[:, None]).ravel()])
    allreduce(buf)
    Q, S = prob.n_pairs, prob.n_scales
    return buf[7 * Q + S:].reshape(-1, 3), buf[7 * Q:7 * Q + S], buf[:7 * Q].reshape(-1, 7)
