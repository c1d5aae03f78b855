"""fp32-vs-fp64 sweep of the factorization's trailing updates (BASELINE config C5's "fp32 vs fp64
tolerance sweep"): the same LM run with deftri_set_factor_precision 0 (fp64, the
reference's arithmetic) and 1 (fp32 MFMA Schur updates), per regime and size; reports the trial
counts, the chi2 trajectory deviation, the reprojection RMSE of the solved map (calculatePixelsStandDev,
the north-star quantity, bar 1e-4 px) and ms per trial.

    python tools/precision_sweep.py > profiles/r02_precision_sweep.json
"""
import copy
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
from deftri import capi, metrics, sim  # noqa: E402

REGIMES = {
    "simulation": dict(kb8=sim.DRUNKARD_KB8, rep=1.0, arap=2e5, sigma=np.float32(0.003)),
    "drunkard": dict(kb8=sim.DRUNKARD_KB8, rep=1.0, arap=1e7, sigma=np.float32(0.3) / np.float32(1000.0)),
    "realcolon": dict(kb8=sim.REALCOLON_KB8, rep=1.0, arap=0.1, sigma=np.float32(0.001) / np.float32(1000.0)),
}


def run(ctx, p, m, n_it, f32):
    ctx.set_factor_precision(f32)
    ctx.upload(p)
    t0 = time.perf_counter()
    r = ctx.solve_lm(n_it, analytic=False)
    dt = time.perf_counter() - t0
    pts, _, _ = ctx.download()
    mm = copy.deepcopy(m)
    metrics.apply_solution(mm, list(p.point_ids), pts)
    rms = metrics.pixels_stand_dev(mm)
    return r, rms, 1e3 * dt / max(r["trials_total"], 1)


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [400, 10000, 100000]
    out = {"what": "fp32 vs fp64 trailing updates (deftri_set_factor_precision)", "cases": []}
    ctx = capi.Context(0)
    ctx.set_lm_lanes(1)
    n_it = 10
    for regime, r in REGIMES.items():
        for n in sizes:
            if regime != "simulation" and n > 10000:
                continue
            m, _ = sim.simulate_two_view(n=n, seed=5, kb8=r["kb8"], scale_scene=True, compact=True)
            p = capi.Context(-1).build_graph(m, r["rep"], r["arap"], np.float32(r["sigma"]))
            r64, rms64, ms64 = run(ctx, p, m, n_it, 0)
            r32, rms32, ms32 = run(ctx, p, m, n_it, 1)
            c64, c32 = np.array(r64["chi2_iter"]), np.array(r32["chi2_iter"])
            k = min(len(c64), len(c32))
            case = {"regime": regime, "correspondences": n, "unknowns": p.n_unknowns, "iterations": n_it,
                    "fp64": {"trials": r64["trials_total"], "chi2_final": r64["chi2_final"], "rms_px": rms64["desv"],
                             "ms_per_trial": ms64},
                    "fp32_updates": {"trials": r32["trials_total"], "chi2_final": r32["chi2_final"],
                                     "rms_px": rms32["desv"], "ms_per_trial": ms32},
                    "chi2_max_rel_dev": float(np.max(np.abs(c32[:k] - c64[:k]) / np.abs(c64[:k]))) if k else None,
                    "rms_delta_px": abs(rms32["desv"] - rms64["desv"])}
            case["rms_delta_px"] = float(case["rms_delta_px"])
            case["within_1e-4_px"] = bool(case["rms_delta_px"] < 1e-4)
            print(json.dumps(case), file=sys.stderr, flush=True)
            out["cases"].append(case)
    ctx.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
