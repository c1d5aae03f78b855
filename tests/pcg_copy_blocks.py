"""Evidence for DESIGN.md §8 "next" item 1 (a preconditioner coupling the keyframe copies of a mesh
vertex).  Test infrastructure (uses the oracle's assembled H); run by hand:

    python tests/pcg_copy_blocks.py 10000 30000 > profiles/r02d_pcg_copy_blocks.txt

Two-view benchmark scene at n correspondences, the dampings the LM visits (7e-3, 0.1, 1 x max diag H,
tests/pcg_evidence.py --observed): CG iterations to relative residual 1e-8 / 1e-10 / 1e-12 with the
block-Jacobi preconditioner the device uses (3x3 point blocks) and with 6x6 blocks pairing each point
with its other keyframe's copy (the points an ARAP edge holds at roles 0/2 and 1/3).
"""
import sys, json, time
import numpy as np, scipy.sparse as sp
import pathlib
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests")); sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
import pcg_evidence as pe
from deftri import sim
from oracle import oracle

def group_inv(A, groups):
    rows, cols, vals = [], [], []
    Ac = A.tocsr()
    for g in groups:
        g = np.asarray(g)
        B = Ac[g][:, g].toarray()
        Bi = np.linalg.inv(B)
        r, c = np.meshgrid(g, g, indexing="ij")
        rows.append(r.ravel()); cols.append(c.ravel()); vals.append(Bi.ravel())
    n = A.shape[0]
    return sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n))

for n in [int(a) for a in sys.argv[1:]]:
    p = sim.two_view_problem(n, 1)
    ri, ci, v = oracle.hessian_coo(p, analytic=False)
    N = p.n_unknowns
    H = sp.csr_matrix((v, (ri, ci)), shape=(N, N))
    b, _, _ = oracle.linearize(p, analytic=False)
    P0 = 6 * p.n_pairs + p.n_scales
    ap = p.arap_pts
    partner = -np.ones(p.n_points, np.int64)
    for a, c in ((0, 2), (1, 3)):
        partner[ap[:, a]] = ap[:, c]; partner[ap[:, c]] = ap[:, a]
    print("unpaired", int((partner < 0).sum()), "n_points", p.n_points, file=sys.stderr)
    base = [list(range(6 * i, 6 * i + 6)) for i in range(p.n_pairs)] + [[6 * p.n_pairs + s] for s in range(p.n_scales)]
    g3 = base + [list(range(P0 + 3 * i, P0 + 3 * i + 3)) for i in range(p.n_points)]
    seen = np.zeros(p.n_points, bool); g6 = list(base)
    for i in range(p.n_points):
        if seen[i]: continue
        j = partner[i]
        if j >= 0 and not seen[j]:
            g6.append(list(range(P0 + 3 * i, P0 + 3 * i + 3)) + list(range(P0 + 3 * j, P0 + 3 * j + 3))); seen[j] = True
        else:
            g6.append(list(range(P0 + 3 * i, P0 + 3 * i + 3)))
        seen[i] = True
    dmax = np.abs(H.diagonal()).max()
    for f in (7e-3, 0.1, 1.0):
        A = (H + f * dmax * sp.identity(N, format="csr")).tocsr()
        x_ref = oracle.damped_solve(p, f * dmax, b, analytic=False)
        r3 = pe.pcg(A, b, group_inv(A, g3), x_ref, [1e-8, 1e-10, 1e-12], 3000)
        r6 = pe.pcg(A, b, group_inv(A, g6), x_ref, [1e-8, 1e-10, 1e-12], 3000)
        print(n, f, "3x3", {k: v["iterations"] for k, v in r3.items()}, "6x6", {k: v["iterations"] for k, v in r6.items()}, flush=True)
