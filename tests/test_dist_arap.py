"""Point-sharded ARAP plan (DistPlan, csrc/symbolic.cpp) on the CPU: world_size-2 gloo ranks run the
host emulation of their part of the multifrontal damped solve (deftri_debug_plan_solve_dist: the
device kernels' task lists and the cross-rank transfers — packed contribution blocks, forward-update
vectors, boundary solutions — through the gloo transport).  Each rank's system is the partial one
its owned edges produce (H_q = sum of J_e^T J_e over them, random per-edge Jacobians on the real
ARAP / reprojection / depth sparsity of g2oBundleAdjustment.cc:765-953), so the test also checks
the edge ownership and the redirection of remote-block contributions.  The gathered solution must
solve the full damped system to backward error < 1e-14 and match the single-rank plan."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp


def _problem():
    from deftri import capi, sim
    m, _ = sim.simulate_two_view(n=260, seed=21)
    host = capi.Context(-1)
    p = host.build_graph(m, 1.0, 2e5, np.float32(0.003))
    host.close()
    return p


def _edge_systems(p, seed=5):
    """Per-edge (dof indices, J rows, residual) with random J on each edge's vertex blocks."""
    rng = np.random.default_rng(seed)
    Q, S = p.n_pairs, p.n_scales
    voff = lambda kind, i: 6 * i if kind == "T" else (6 * Q + i if kind == "s" else 6 * Q + S + 3 * i)
    edges = {"rep": [], "dep": [], "arap": []}
    for e in range(len(p.rep_point)):
        d = [voff("p", p.rep_point[e]) + k for k in range(3)]
        edges["rep"].append((d, rng.normal(size=(2, 3)), rng.normal(size=2)))
    for e in range(len(p.dep_point)):
        d = [voff("p", p.dep_point[e]) + k for k in range(3)] + [voff("s", p.dep_scale[e])]
        edges["dep"].append((d, rng.normal(size=(1, 4)), rng.normal(size=1)))
    for e in range(len(p.arap_pair)):
        d = []
        for q in range(4):
            d += [voff("p", p.arap_pts.reshape(-1, 4)[e, q]) + k for k in range(3)]
        d += [voff("T", p.arap_pair[e]) + k for k in range(6)]
        edges["arap"].append((d, rng.normal(size=(1, 18)) * 1e-2, rng.normal(size=1)))
    return edges


def _assemble(p, edges, masks=None):
    n = p.n_unknowns
    H = np.zeros((n, n)); b = np.zeros(n)
    for kind in ("rep", "dep", "arap"):
        for e, (d, J, r) in enumerate(edges[kind]):
            if masks is not None and not masks[kind][e]:
                continue
            H[np.ix_(d, d)] += J.T @ J
            b[d] += J.T @ r
    return H, b


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deftri import capi
    from deftri import dist as ddist
    p = _problem()
    ctx = capi.Context(-1)
    ctx.dist_set_transport(world, rank, ddist.torch_transport())
    ctx.analyse(p)
    rep, dep, arap = ctx.owned_edges()
    owner = ctx.vertex_owner()
    edges = _edge_systems(p)
    Hq, bq = _assemble(p, edges, {"rep": rep, "dep": dep, "arap": arap})
    lam = 0.37
    x = ctx.debug_plan_solve_dist(Hq, lam, bq)
    q.put((rank, x, owner, rep, dep, arap))
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_damped_solve_gloo(world):
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = 29700 + world * 17 + os.getpid() % 500
    procs = [ctxm.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = {}
    for _ in procs:
        rank, *rest = q.get(timeout=300)
        out[rank] = rest
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    from deftri import capi
    p = _problem()
    edges = _edge_systems(p)
    # every edge is owned by exactly one rank
    for k, key in enumerate(("rep", "dep", "arap")):
        cnt = sum(out[r][2 + k].astype(int) for r in range(world))
        assert np.all(cnt == 1), key
    owner = out[0][1]
    assert all(np.array_equal(out[r][1], owner) for r in range(world))
    assert set(np.unique(owner)) == set(range(world))          # every rank owns part of the graph
    # authoritative dofs per rank -> full solution
    Q, S = p.n_pairs, p.n_scales
    vdim = np.r_[np.full(Q, 6), np.ones(S, int), np.full(p.n_points, 3)]
    dof_owner = np.repeat(owner, vdim)
    x = np.zeros(p.n_unknowns)
    for r in range(world):
        x[dof_owner == r] = out[r][0][dof_owner == r]
    H, b = _assemble(p, edges)
    lam = 0.37
    A = H + lam * np.eye(len(b))
    berr = np.linalg.norm(A @ x - b) / (np.linalg.norm(A, 2) * np.linalg.norm(x))
    assert berr < 1e-14, berr
    # the single-rank plan on the full system
    host = capi.Context(-1)
    host.analyse(p)
    x1 = host.debug_plan_solve(H, lam, b)
    assert np.linalg.norm(x - x1) <= 1e-10 * np.linalg.norm(x1)
    # replicated dofs (boundary of each rank's top front) agree with their owner's values
    for r in range(world):
        xr = out[r][0]
        nz = (xr != 0) & (dof_owner != r)
        assert np.allclose(xr[nz], x[nz], rtol=1e-12, atol=0)
