"""Which ARAP Jacobian columns differ between k_lin_arap<2> and <3> (DEFTRI_ARAP_J_FULL): the
gradient b and diag H of the iterative plan at the initial state, per dof class, in two processes."""
import multiprocessing as mp
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "triangulation-in-deformable-scenes_amd"))


def worker(env, q):
    os.environ.update(env)
    from deftri import capi, sim
    m, _ = sim.simulate_two_view(n=5000, seed=6, scale_scene=True, compact=True)
    host = capi.Context(-1)
    p = host.build_graph(m, 1.0, 2e5, np.float32(0.003))
    host.close()
    with capi.Context(0) as ctx:
        ctx.set_plan("iterative")
        ctx.upload(p)
        b, d = ctx.gradient()
        q.put((np.asarray(b).copy(), np.asarray(d).copy(), 6 * p.tg.shape[0] + np.asarray(p.scales).size))


if __name__ == "__main__":
    cm = mp.get_context("spawn")
    out = []
    for env in ({}, {"DEFTRI_ARAP_J_FULL": "1"}):
        q = cm.Queue()
        pr = cm.Process(target=worker, args=(env, q))
        pr.start()
        out.append(q.get(timeout=300))
        pr.join()
    (b0, d0, hd), (b1, d1, _) = out
    for name, x, y in (("b", b0, b1), ("diag", d0, d1)):
        for cls, sl in (("heavy(T_g)", slice(0, hd)), ("points", slice(hd, None))):
            xa, ya = x[sl], y[sl]
            nd = int((xa.view(np.int64) != ya.view(np.int64)).sum())
            print(name, cls, "differing", nd, "of", xa.size, "max rel", float(np.max(np.abs(xa - ya) / (np.abs(ya) + 1e-300))) if xa.size else 0)
    dif = (b0[hd:].view(np.int64) != b1[hd:].view(np.int64)).reshape(-1, 3)
    print("points b: differing per component", dif.sum(axis=0))
