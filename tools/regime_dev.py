"""Per-variant deviation of the iterative plan's LM run from a committed regime golden (chi2 per
iteration, trials, RMSE), for A/Bs of summation-order changes.

usage: python tools/regime_dev.py NAME SUB [ENV=VAL[,ENV=VAL] ...]   ('-' = no extra env)"""
import json
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))


def one(name, sub):
    import copy
    import numpy as np
    import torch  # noqa: F401
    from deftri import capi, metrics
    from test_regime_goldens import golden, scene
    meta, z = golden(name, sub)
    p, m = scene(meta)
    with capi.Context(0) as c:
        c.set_plan("iterative")
        c.set_lm_lanes(1)
        c.upload(p)
        r = c.solve_lm(meta["n_iterations"], analytic=False)
        pts = c.download()[0]
    a, b = np.array(r["chi2_iter"]), np.array(z["chi2_iter"])
    rel = np.abs(a - b) / np.abs(b)
    m1 = copy.deepcopy(m)
    metrics.apply_solution(m1, list(p.point_ids), pts)
    rms = metrics.pixels_stand_dev(m1)
    return {"max_rel": float(rel.max()), "at": int(rel.argmax()), "trials_same": r["trials_iter"] == list(z["trials_iter"]),
            "rms_dev": abs(rms["desv"] - meta["rms_final"]["desv"])}


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        print("RESULT " + json.dumps(one(sys.argv[2], sys.argv[3])), flush=True)
        sys.exit(0)
    name, sub = sys.argv[1], sys.argv[2]
    for v in sys.argv[3:] or ["-"]:
        env = dict(kv.split("=", 1) for kv in v.split(",")) if v != "-" else {}
        res = subprocess.run([sys.executable, __file__, "--one", name, sub], env=dict(os.environ, **env), capture_output=True,
                             text=True, timeout=600)
        line = [l for l in res.stdout.splitlines() if l.startswith("RESULT ")]
        if res.returncode or not line:
            print(json.dumps({"env": env, "rc": res.returncode, "stderr": res.stderr[-2000:]}), flush=True)
            sys.exit(1)
        print(json.dumps(dict(json.loads(line[0][7:]), env=env)), flush=True)
