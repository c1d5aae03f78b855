"""Evidence for DESIGN.md §8: warm-starting a rejected trial's PCG solve.  Test infrastructure (uses
the oracle's assembled H); run by hand:

    python tests/pcg_warm_start.py 10000 30000 > profiles/r02d_pcg_warm_start.txt

Two-view benchmark scene: the first trial's solve at lambda (f x max diag H, the dampings the LM
visits), then the retry g2o makes after a rejection at nu x lambda (nu = 2, 4), from x = 0 (cold),
from the first trial's solution (warm) and from its best multiple (scaled warm); CG iterations to
relative residual 1e-12 with the device's block-Jacobi preconditioner.
"""
import sys
import numpy as np, scipy.sparse as sp
import pathlib
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests")); sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
import pcg_evidence as pe
from deftri import sim
from oracle import oracle

def pcg(A, b, M, x0, tol, max_it=3000):
    x = x0.copy(); r = b - A @ x; z = M @ r; p = z.copy(); rz = r @ z; nb = np.linalg.norm(b)
    if np.linalg.norm(r) <= tol * nb: return x, 0
    for it in range(1, max_it + 1):
        Ap = A @ p; alpha = rz / (p @ Ap); x += alpha * p; r -= alpha * Ap
        if np.linalg.norm(r) <= tol * nb: return x, it
        z = M @ r; rzn = r @ z; p = z + (rzn / rz) * p; rz = rzn
    return x, None

for n in [int(a) for a in sys.argv[1:]]:
    p = sim.two_view_problem(n, 1)
    ri, ci, v = oracle.hessian_coo(p, analytic=False)
    N = p.n_unknowns
    H = sp.csr_matrix((v, (ri, ci)), shape=(N, N))
    b, _, _ = oracle.linearize(p, analytic=False)
    dims = [(6, p.n_pairs), (1, p.n_scales), (3, p.n_points)]
    dmax = np.abs(H.diagonal()).max()
    for f in (7e-3, 0.1):
        lam = f * dmax
        A = (H + lam * sp.identity(N, format="csr")).tocsr()
        x1, i1 = pcg(A, b, pe.block_jacobi(A, dims), np.zeros(N), 1e-12)
        for nu in (2.0, 4.0):
            A2 = (H + nu * lam * sp.identity(N, format="csr")).tocsr(); M2 = pe.block_jacobi(A2, dims)
            _, c = pcg(A2, b, M2, np.zeros(N), 1e-12)
            _, w = pcg(A2, b, M2, x1, 1e-12)
            # scaled warm start: x1 minimises along the previous solution direction
            Ax = A2 @ x1; s = (x1 @ b) / (x1 @ Ax)
            _, ws = pcg(A2, b, M2, s * x1, 1e-12)
            print(n, f, nu, "first", i1, "cold", c, "warm", w, "scaled-warm", ws, flush=True)
