"""GPU debug: the C++ adapter's bundleAdjustment against deftri.ba on the same map (chi2 reports)."""
import copy, pathlib, subprocess, sys
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "tests"), str(ROOT / "triangulation-in-deformable-scenes_amd")]
import numpy as np
from adapter_io import read_state, write_map
from deftri import ba
m, _ = ba.simulate_ba_map(n=300, k=4, seed=5, outliers=0.05, visibility=0.9)
out = ROOT / "gpurun_out" / "r06c"
out.mkdir(parents=True, exist_ok=True)
mm = copy.deepcopy(m)
write_map(out / "ba.bin", mm)
prob, meta = ba.build_ba_graph([mm.keyframes[k] for k in mm.kf_order()])
print("py order", mm.kf_order(), "poses", prob.poses.tolist()[:2], "n_edges", prob.n_edges, "n_points", prob.n_points)
rep = {}
ba.bundleAdjustment(mm, report=rep)
print("py chi2", rep["chi2_initial"], rep["chi2_final"], rep["iterations"], rep["trials_total"])
r = subprocess.run([str(ROOT / "adapter/build/adapter_driver"), str(out / "ba.bin"), str(out / "ba.out"), "ba"],
                   capture_output=True, text=True)
print("rc", r.returncode, r.stderr[-2000:])
s = read_state(out / "ba.out")
print("cpp chi2", s["extra"])
for pid in list(mm.map_points)[:3]:
    print(pid, s["points"][pid], mm.map_points[pid].position)
