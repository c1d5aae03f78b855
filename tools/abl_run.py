"""Kernel-time probe for build variants (ablations / A/B): the C2 problem (or N_CORR), a few LM
iterations on the library DEFTRI_LIB names; run under rocprofv3 --kernel-trace, then
tools/abl_run.py --summ DIR prints per-kernel median durations of the non-early-out launches.

usage: python tools/abl_run.py N_CORR N_IT
       python tools/abl_run.py --summ TRACE_DIR [MIN_US]"""
import csv
import re
import glob
import json
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent

if sys.argv[1] == "--summ":
    files = glob.glob(sys.argv[2] + "/**/*kernel_trace.csv", recursive=True)
    lo = float(sys.argv[3]) if len(sys.argv) > 3 else 8.0
    d = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            n = row["Kernel_Name"]
            us = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
            for k in ("k_sp_tile", "k_sp_tupd", "k_lin_arap", "k_sp_glin_rows", "k_sp_glin_blocks", "k_trial_eval", "k_sp_setup"):
                if re.search(r"\b" + k + r"[<(I]", n):
                    d.setdefault(k, []).append(us)
    print(json.dumps({k: {"n": len(v), "n_full": len([x for x in v if x >= lo]),
                          "median_full_us": round(statistics.median([x for x in v if x >= lo] or [0]), 2),
                          "min_us": round(min(v), 2)} for k, v in sorted(d.items())}))
    sys.exit(0)

sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
import torch  # noqa: F401,E402
from deftri import capi, sim  # noqa: E402
p = sim.two_view_problem(int(sys.argv[1]), 1)
with capi.Context(0) as ctx:
    ctx.set_plan("iterative")
    ctx.upload(p)
    r = ctx.solve_lm(int(sys.argv[2]), analytic=False)
    print(json.dumps({"trials": r["trials_iter"], "pcg_its": r["pcg_iterations"]}))
