"""Stage times of the drop-in arapOptimization call (bench.py's end_to_end: cold, warm, next round) at
N_CORR correspondences: run with DEFTRI_CALL_TIMING=1 DEFTRI_PLAN_TIMING=1 DEFTRI_GRAPH_TIMING=1
DEFTRI_UPLOAD_TIMING=1 to get the library's per-stage lines on stderr.

usage: python tools/e2e_timing.py [N_CORR]"""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
import torch  # noqa: F401,E402
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
p, m = bench.build_problem(n, 1)
print(json.dumps(bench.end_to_end(0, m, lambda c: c.set_plan("auto"))), flush=True)
