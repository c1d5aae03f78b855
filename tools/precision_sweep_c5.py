"""C5's fp32-vs-fp64 sweep on the timed path (BASELINE configs[4]): the iterative
plan's product with the ARAP Jacobians stored in fp64 (the reference's precision) and in fp32
(deftri_set_jacobian_storage 1: b, the preconditioner, every vector and every reduction stay fp64).

Per scene, the same initial state, N LM iterations (g2o numeric Jacobians): trial counts, the largest
relative chi2 deviation per iteration, the reprojection RMSE of the solved map
(calculatePixelsStandDev on the device, Geometry.cc:370-498) and its delta to the fp64 run, the
product's algorithmic bytes per CG iteration and its profiled time.

usage: python tools/precision_sweep_c5.py OUT.json [n_per_kf] [iterations] [scene ...]
  scenes: c5w (Realcolon 20 KFs, 19 consecutive pairs), c5a (Realcolon 20 KFs, all 190 pairs),
          c4 (Drunkard 8 KFs, all 28 pairs)
"""
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
from deftri import capi, sim  # noqa: E402

SCENES = {
    "c5w": dict(k=20, kb8=sim.REALCOLON_KB8, w=(1.0, 0.1, 1e-6), window=1),
    "c5a": dict(k=20, kb8=sim.REALCOLON_KB8, w=(1.0, 0.1, 1e-6), window=0),
    "c4": dict(k=8, kb8=sim.DRUNKARD_KB8, w=(1.0, 1e7, 0.3), window=0),
}


def apply(am, ids, pts, n):
    """write the solved points (graph order, MapPoint id k * n + i) into the ArrayMap's keyframes"""
    ids = np.asarray(ids)
    k, i = ids // n, ids % n
    for kk in range(len(am.kfs)):
        sel = k == kk
        am.kfs[kk]["pos"][i[sel]] = pts[sel].astype(np.float32)


def run(name, n, n_it):
    sc = SCENES[name]
    t0 = time.time()
    am = sim.multi_view_arrays(n=n, k=sc["k"], seed=1, kb8=sc["kb8"])
    host = capi.Context(-1)
    if sc["window"]:
        host.set_pair_window(sc["window"])
    rep, arap, sig = sc["w"]
    prob = host.build_graph(am, rep, arap, np.float32(sig))
    init = [kf["pos"].copy() for kf in am.kfs]
    print(f"{name} {n}: built in {time.time() - t0:.1f} s: {prob.summary()}", flush=True)
    out = {"scene": name, "n_per_kf": n, "keyframes": sc["k"], "pairs": prob.n_pairs, "unknowns": prob.n_unknowns,
           "arap_edges": len(prob.arap_pair), "iterations": n_it, "runs": {}}
    ctx = capi.Context(0)
    rms = {}
    for fp32 in (0, 1):
        ctx.set_plan("iterative")
        ctx.set_jacobian_storage(fp32)
        ctx.upload(prob)
        info = ctx.plan_info()
        t = time.time()
        r = ctx.solve_lm(n_it, analytic=False)
        dt = time.time() - t
        pts, _, _ = ctx.download()
        st = ctx.profile_trial(r["lambda_final"])
        its = max(st["sp_phase2"]["launches"], 1)
        prod_us = 1e3 * (st["sp_phase1"]["ms"] + st["sp_phase2"]["ms"]) / its
        for kk, kf in enumerate(am.kfs):
            kf["pos"][:] = init[kk]
        apply(am, prob.point_ids, pts, n)
        pe = ctx.pixels_stand_dev(am)
        rms[fp32] = pe
        out["runs"]["fp32" if fp32 else "fp64"] = {
            "trials": r["trials_total"], "chi2_iter": r["chi2_iter"], "chi2_final": r["chi2_final"],
            "pcg_trials": r["pcg_trials"], "pcg_failed": r["pcg_fallbacks"], "cg_iterations": r["pcg_iterations"],
            "ms_per_iteration": round(1e3 * dt / max(r["iterations"], 1), 3),
            "product_bytes_per_cg_iteration": info["product_bytes"], "product_us_profiled": round(prod_us, 2),
            "rmse_desv": pe["desv"], "rmse_desvc1": pe["desvc1"], "rmse_desvc2": pe["desvc2"]}
        print(name, "fp32" if fp32 else "fp64", json.dumps(out["runs"]["fp32" if fp32 else "fp64"])[:400], flush=True)
    a, b = np.array(out["runs"]["fp32"]["chi2_iter"]), np.array(out["runs"]["fp64"]["chi2_iter"])
    m = min(len(a), len(b))
    out["chi2_max_rel_dev"] = float(np.max(np.abs(a[:m] - b[:m]) / np.abs(b[:m])))
    out["rmse_delta_px"] = {k: abs(rms[1][k] - rms[0][k]) for k in ("desv", "desvc1", "desvc2")}
    out["same_trials"] = out["runs"]["fp32"]["trials"] == out["runs"]["fp64"]["trials"]
    out["within_1e-4_px"] = max(out["rmse_delta_px"].values()) < 1e-4
    ctx.close()
    return out


def main():
    dst = pathlib.Path(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
    n_it = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    names = sys.argv[4:] or ["c5w"]
    res = [run(nm, n if nm != "c5a" else min(n, 20000), n_it) for nm in names]
    dst.parent.mkdir(parents=True, exist_ok=True)
    dst.write_text(json.dumps(res, indent=1))
    for r in res:
        print(r["scene"], r["n_per_kf"], "same trials", r["same_trials"], "chi2 dev", r["chi2_max_rel_dev"],
              "rmse delta", r["rmse_delta_px"], flush=True)


if __name__ == "__main__":
    main()
