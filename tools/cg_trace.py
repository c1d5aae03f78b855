"""Per-trial CG iteration counts against lambda for a C2 LM run (verbose solver log): the data behind
the CG-count guess of each trial's queued chain (spcg_solver.cpp)."""
import os, sys, pathlib, re, subprocess, json
ROOT = pathlib.Path(__file__).resolve().parent.parent
if len(sys.argv) > 1 and sys.argv[1] == "--one":
    sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
    import torch  # noqa
    from deftri import capi, sim
    p = sim.two_view_problem(int(sys.argv[2]), 1)
    with capi.Context(0) as ctx:
        ctx.set_plan("iterative")
        ctx.upload(p)
        r = ctx.solve_lm(int(sys.argv[3]), verbose=True)
        print("RESULT " + json.dumps({"trials": r["trials_iter"], "pcg": r["pcg_iterations"], "cont": r["pcg_continuations"]}), flush=True)
    sys.exit(0)
res = subprocess.run([sys.executable, __file__, "--one", sys.argv[1] if len(sys.argv) > 1 else "100000", "25"],
                     capture_output=True, text=True, timeout=600)
trials = re.findall(r"pcg lambda ([0-9.e+-]+) iterations (\d+) (\S+)", res.stderr)
for lam, its, ok in trials:
    print(lam, its, ok)
print([l for l in res.stdout.splitlines() if l.startswith("RESULT")])
