"""Dev helper: time the device LM on a synthetic two-view scene of n correspondences."""
import sys, time, json, pathlib
import numpy as np
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
from deftri import sim, capi
n = int(sys.argv[1]); nit = int(sys.argv[2])
t = time.time(); m, gt = sim.simulate_two_view(n=n, seed=1, scale_scene=True, compact=True)
host = capi.Context(-1); prob = host.build_graph(m, 1.0, 2e5, np.float32(3.0 / 1000))
print("built", time.time() - t, prob.summary(), flush=True)
ctx = capi.Context(0)
t = time.time(); ctx.upload(prob); print("upload+analyse s", time.time() - t, flush=True)
r = ctx.solve_lm(1, analytic=True)   # warm-up
ctx.reset_state()
t = time.time(); r = ctx.solve_lm(nit, analytic=True); dt = time.time() - t
print(json.dumps({k: r[k] for k in ("chi2_initial", "chi2_final", "iterations", "trials_total", "ms_total", "ms_linearize", "ms_factor", "ms_solve", "ms_update", "n_fronts", "n_levels", "factor_flops", "nnz_factor")}), flush=True)
print("wall s", dt, "ms/iter", 1e3 * dt / max(r["iterations"], 1), "factor TF/s", r["factor_flops"] * r["trials_total"] / (r["ms_factor"] * 1e-3) / 1e12)
