"""Dev helper (GPU): multi-view damped-solve accuracy vs the oracle's LDL^T and dense LAPACK."""
import sys, pathlib
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "triangulation-in-deformable-scenes_amd"), str(ROOT)]
import numpy as np
from deftri import capi, sim
from oracle import oracle
m, _ = sim.simulate_multi_view(n=200, k=3, seed=4)
p = capi.Context(-1).build_graph(m, 1.0, 2e5, np.float32(0.003))
ctx = capi.Context(0); ctx.upload(p)
b_ref, H, _ = oracle.linearize(p, analytic=True, dense=True)
for lr in (1e-5, 1e-3, 1e-1):
    lam = lr * np.abs(np.diag(H)).max()
    x = ctx.damped_solve(lam, b_ref)
    A = H + lam * np.eye(len(b_ref))
    xr = np.linalg.solve(A, b_ref)
    xo = oracle.damped_solve(p, lam, b_ref)
    print(f"lam_rel {lr:g}: bwd {np.linalg.norm(A @ x - b_ref) / (np.linalg.norm(A, 2) * np.linalg.norm(x)):.2e} "
          f"rel vs lapack {np.linalg.norm(x - xr) / np.linalg.norm(xr):.2e} rel vs oracle {np.linalg.norm(x - xo) / np.linalg.norm(xo):.2e} "
          f"oracle vs lapack {np.linalg.norm(xo - xr) / np.linalg.norm(xr):.2e} cond {np.linalg.cond(A):.2e}")
r = ctx.solve_lm(5, analytic=True); ref = oracle.solve_lm(p, 5, analytic=True)["report"]
print(np.array(r["chi2_iter"]) / np.array(ref["chi2_iter"]) - 1, r["trials_iter"], ref["trials_iter"])
