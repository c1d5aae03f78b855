"""The iterative plan's point-sharded product decomposition (csrc/spcg.h; host emulation
deftri_debug_sp_product, no GPU) against a direct numpy product.

For an all-pairs 8-keyframe graph (BASELINE C3/C4 shape, g2oBundleAdjustment.cc:640-645) and a
two-view graph, with random per-edge Jacobians and weights: q = (sum_e J_e^T W_e J_e + lambda I) p.
World sizes 1, 2, 3 run as gloo processes: each rank reads only its own rows of p, receives its halo
rows through the transport (the device exchange's send / receive order), all-reduces its owned edges'
global-vertex partials; the ranks' rows, summed, must equal the single product to 1e-12 relative.
Also checked: the row partition covers every point once and each ARAP edge is owned by exactly one rank."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp


def _problem(kind):
    from deftri import capi, sim
    if kind == "mv":
        m, _ = sim.simulate_multi_view(n=150, k=8, seed=3)
        w = (1.0, 1e7, np.float32(0.3))
    else:
        m, _ = sim.simulate_two_view(n=2000, seed=5, scale_scene=True, compact=True)
        w = (1.0, 2e5, np.float32(0.003))
    host = capi.Context(-1)
    p = host.build_graph(m, *w)
    host.close()
    return p


def _random_lin(p, seed=0):
    rng = np.random.default_rng(seed)
    E, R, D = len(p.arap_pair), len(p.rep_point), len(p.dep_point)
    return (rng.normal(size=(E, 18)), rng.uniform(0.5, 2.0, E), rng.normal(size=(R, 6)), rng.uniform(0.5, 2.0, R),
            rng.normal(size=(D, 4)), rng.uniform(0.5, 2.0, D), rng.normal(size=p.n_unknowns))


def _reference(p, Ja, Wa, Jr, Wr, Jd, Wd, lam, x):
    Q, S = p.n_pairs, p.n_scales
    hd = 6 * Q + S
    q = lam * x.copy()
    pt = lambda idx: hd + 3 * np.asarray(idx)[:, None] + np.arange(3)[None, :]
    # ARAP: s = W J v over (4 points, T_g)
    cols = np.concatenate([pt(p.arap_pts[:, k]) for k in range(4)] + [6 * p.arap_pair[:, None] + np.arange(6)[None, :]], 1)
    s = Wa * np.einsum("ej,ej->e", Ja, x[cols])
    np.add.at(q, cols, Ja * s[:, None])
    # reprojection: 2 x 3 on the point
    c = pt(p.rep_point)
    J2 = Jr.reshape(-1, 2, 3)
    t = np.einsum("erk,ek->er", J2, x[c]) * Wr[:, None]
    np.add.at(q, c, np.einsum("erk,er->ek", J2, t))
    # depth: point + scale
    cd = np.concatenate([pt(p.dep_point), (6 * Q + p.dep_scale)[:, None]], 1)
    s = Wd * np.einsum("ej,ej->e", Jd, x[cd])
    np.add.at(q, cd, Jd * s[:, None])
    return q


def _worker(rank, world, port, kind, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deftri import capi
    from deftri import dist as ddist
    p = _problem(kind)
    lin = _random_lin(p)
    with capi.Context(-1) as ctx:
        if world > 1:
            ctx.dist_set_transport(world, rank, ddist.torch_transport())
        qv, st = ctx.debug_sp_product(p, *lin[:6], 0.37, lin[6])
    q.put((rank, qv, st))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["mv", "tv"])
@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_product_matches_direct(kind, world):
    cm = mp.get_context("spawn")
    q = cm.Queue()
    port = 29600 + 17 * world + (1 if kind == "mv" else 0) + os.getpid() % 400
    procs = [cm.Process(target=_worker, args=(r, world, port, kind, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = {}
    for _ in procs:
        r, qv, st = q.get(timeout=300)
        out[r] = (qv, st)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p = _problem(kind)
    lin = _random_lin(p)
    ref = _reference(p, *lin[:6], 0.37, lin[6])
    hd = 6 * p.n_pairs + p.n_scales
    total = np.zeros_like(ref)
    covered = np.zeros(p.n_points, int)
    owned = 0
    for r in range(world):
        qv, st = out[r]
        np.testing.assert_allclose(qv[:hd], ref[:hd], rtol=1e-12, atol=1e-12 * np.abs(ref[:hd]).max())
        rows = np.any(qv[hd:].reshape(-1, 3) != 0, 1)
        covered += rows
        total[hd:] += qv[hd:]
        owned += st[3]
        assert st[0] > 0 and st[2] >= st[3]
        if world > 1:
            assert st[1] > 0                        # a halo exists between mesh-adjacent shards
        else:
            assert st[1] == 0 and st[2] == st[3] == len(p.arap_pair)
    assert owned == len(p.arap_pair)
    assert covered.max() == 1                       # no point row produced by two ranks
    total[:hd] = ref[:hd]
    np.testing.assert_allclose(total, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())
