"""Dev helper: C2 LM with a given lane count (for rocprofv3 kernel traces of the speculative lanes)."""
import sys, time, pathlib
import numpy as np
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
from deftri import sim, capi
n, lanes, nit = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
m, gt = sim.simulate_two_view(n=n, seed=1, scale_scene=True, compact=True)
prob = capi.Context(-1).build_graph(m, 1.0, 2e5, np.float32(3.0 / 1000))
ctx = capi.Context(0)
ctx.upload(prob)
ctx.set_lm_lanes(lanes)
ctx.solve_lm(1, analytic=True)
ctx.reset_state()
t = time.time(); r = ctx.solve_lm(nit, analytic=True); dt = time.time() - t
print("lanes", r["lanes"], "iters", r["iterations"], "trials", r["trials_total"], "executed", r["trials_executed"],
      "ms/iter", 1e3 * dt / max(r["iterations"], 1), "trials_iter", r["trials_iter"], flush=True)
