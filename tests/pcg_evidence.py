"""Evidence for DESIGN.md §2's choice of a direct factorization over the matrix-free PCG SURVEY §8
sketched.  Test infrastructure (uses the oracle's assembled H); run by hand:

    python tests/pcg_evidence.py 10000 30000 100000 > profiles/r02_pcg_evidence.json
    python tests/pcg_evidence.py --observed 10000 > profiles/r02_pcg_evidence_observed.json

For the two-view benchmark scene at n correspondences: the damped system (H + lam I) dx = b of the
first LM iteration (lam = tau * max diag H, tau = 1e-5, g2o's initial damping) and of later, weaker
dampings (1e-7 and 1e-9 of max diag H), solved by conjugate gradients with the block-Jacobi preconditioner
(one block of H + lam I per vertex: 6x6 T_g, 1x1 scale, 3x3 point; at most 10000 iterations) — the preconditioner the PCG plan named —
against the direct solve (the oracle's sparse LDL^T).  Reported: CG iterations to relative residual
1e-4 / 1e-6 / 1e-8 / 1e-10 and the relative error of the step at those points.
"""
import json
import pathlib
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
sys.path.insert(0, str(ROOT))
from deftri import sim  # noqa: E402
from oracle import oracle  # noqa: E402


def block_jacobi(H, dims):
    """Sparse inverse of the vertex-block diagonal of H."""
    rows, cols, vals = [], [], []
    off = 0
    Hc = H.tocsr()
    for d, cnt in dims:
        for _ in range(cnt):
            B = Hc[off:off + d, off:off + d].toarray()
            Bi = np.linalg.inv(B)
            r, c = np.meshgrid(np.arange(off, off + d), np.arange(off, off + d), indexing="ij")
            rows.append(r.ravel()); cols.append(c.ravel()); vals.append(Bi.ravel())
            off += d
    n = H.shape[0]
    return sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n))


def pcg(A, b, M, x_ref, tols, max_it):
    """Preconditioned CG from x = 0; iteration count and step error at each residual tolerance."""
    x = np.zeros_like(b)
    r = b.copy()
    z = M @ r
    p = z.copy()
    rz = r @ z
    nb = np.linalg.norm(b)
    nref = np.linalg.norm(x_ref)
    out, t_i = {}, 0
    for it in range(1, max_it + 1):
        Ap = A @ p
        alpha = rz / (p @ Ap)
        x += alpha * p
        r -= alpha * Ap
        res = np.linalg.norm(r) / nb
        while t_i < len(tols) and res <= tols[t_i]:
            out[f"{tols[t_i]:.0e}"] = {"iterations": it, "step_rel_error": float(np.linalg.norm(x - x_ref) / nref)}
            t_i += 1
        if t_i == len(tols):
            break
        z = M @ r
        rz_new = r @ z
        p = z + (rz_new / rz) * p
        rz = rz_new
    for t in tols[t_i:]:
        out[f"{t:.0e}"] = {"iterations": None, "after_max_iterations": max_it,
                           "residual": float(res), "step_rel_error": float(np.linalg.norm(x - x_ref) / nref)}
    return out


OBSERVED = False


def main():
    global OBSERVED
    args = sys.argv[1:]
    if "--observed" in args:
        OBSERVED = True
        args.remove("--observed")
    sizes = [int(a) for a in args] or [10000]
    res = {"what": __doc__.strip().splitlines()[0], "cases": []}
    for n in sizes:
        t0 = time.time()
        p = sim.two_view_problem(n, 1)
        ri, ci, v = oracle.hessian_coo(p, analytic=False)
        N = p.n_unknowns
        H = sp.csr_matrix((v, (ri, ci)), shape=(N, N))
        b, _, _ = oracle.linearize(p, analytic=False)
        dims = [(6, p.n_pairs), (1, p.n_scales), (3, p.n_points)]   # problem order: [T_g][scales][points]
        assert sum(d * c for d, c in dims) == N, (dims, N)
        dmax = np.abs(H.diagonal()).max()
        case = {"correspondences": n, "unknowns": N, "nnz_H": int(H.nnz),
                "diag_H_range": [float(np.abs(H.diagonal()).min()), float(dmax)]}
        # g2o starts at tau * max diag H (tau = 1e-5) and each accepted trial scales lambda by 1/3..2/3:
        # after ~10 / ~20 accepted iterations it is 1e-2 / 1e-4 of the start or less
        lams = (("initial", 1e-5 * dmax), ("later_1e-7", 1e-7 * dmax), ("later_1e-9", 1e-9 * dmax))
        if OBSERVED:
            # the dampings g2o's LM actually visits on this scene: after the first iteration's
            # rejections lambda sits between ~7e-3 and ~1.7 of max diag H (oracle LM, 25 iterations
            # at 10k correspondences: 1.0e15 .. 2.6e17 against max diag 1.5e17)
            lams = tuple((f"observed_{f:g}", f * dmax) for f in (7e-3, 0.1, 1.0))
        for name, lam in lams:
            A = (H + lam * sp.identity(N, format="csr")).tocsr()
            M = block_jacobi(A, dims)
            t1 = time.time()
            x_ref = oracle.damped_solve(p, lam, b, analytic=False)
            t_direct = time.time() - t1
            t1 = time.time()
            out = pcg(A, b, M, x_ref, [1e-4, 1e-6, 1e-8, 1e-10] + ([1e-12] if OBSERVED else []), 10000)
            case[name] = {"lambda": lam, "cpu_direct_s": t_direct, "cpu_pcg_s": time.time() - t1, "pcg": out}
            print(n, name, json.dumps(out), file=sys.stderr, flush=True)
        case["wall_s"] = time.time() - t0
        res["cases"].append(case)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
