"""The oracle's own spread on a regime golden: the same LM run with other elimination orders of the
exact LDL^T step (the oracle's own nested dissection), chi2 per iteration against the committed golden
(which eliminates in the host analysis' nested-dissection order).  Test infrastructure only.

usage: python tools/oracle_spread.py NAME [SUB [MODES]]   (MODES: oracle_nd,edge_rev)
       python tools/oracle_spread.py c2_realcolon     (the C2 Realcolon golden, tests/golden/c2_realcolon:
                                                       about an hour of one core)"""
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests" / "golden"))
sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
sys.path.insert(0, str(ROOT))
from make_regime_goldens import scene, N_IT   # noqa: E402
from oracle import oracle                      # noqa: E402

name, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "regimes")
if name == "c2_realcolon":
    from make_c2_golden import REGIMES as C2R, N_CORR, SEED
    from deftri import capi, sim
    d = ROOT / "tests" / "golden" / name
    meta = json.loads((d / "expected_c2.json").read_text())
    z = np.load(d / "expected_c2.npz")
    rep, arap, sig, kb8 = C2R["realcolon"]
    p = sim.two_view_problem(N_CORR, SEED, rep, arap, sig, kb8=getattr(sim, kb8))
    N_IT = meta["n_iterations"]
else:
    d = ROOT / "tests" / "golden" / sub
    meta = json.loads((d / f"{name}.json").read_text())
    z = np.load(d / f"{name}.npz")
    p, m, host = scene(name, meta["n_corr"], meta["seed"])
    host.analyse(p)
# the modes: "oracle_nd" the oracle's own nested dissection instead of the golden's elimination order;
# "edge_rev" the golden's order, every edge type's chi2 sums and H / b accumulation walked backwards
modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["oracle_nd"]
golden_order = None
if "edge_rev" in modes:
    from deftri import capi as _capi
    with _capi.Context(-1) as hc:
        hc.analyse(p)
        golden_order = hc.vertex_order()
for label in modes:
    oracle.set_vertex_order(None if label == "oracle_nd" else golden_order)
    oracle.set_edge_order(label == "edge_rev")
    r = oracle.solve_lm(p, N_IT, analytic=False)["report"]
    oracle.set_vertex_order(None)
    oracle.set_edge_order(False)
    a, b = np.array(r["chi2_iter"]), np.array(z["chi2_iter"])
    rel = np.abs(a - b) / np.abs(b)
    lam_ref = meta.get("lambda_final")
    lam_rel = abs(r["lambda_final"] - lam_ref) / abs(lam_ref) if lam_ref else None
    print(json.dumps({"order": label, "max_rel": float(rel.max()), "at": int(rel.argmax()), "lambda_final_rel": lam_rel,
                      "trials_same": list(r["trials_iter"]) == list(z["trials_iter"])}), flush=True)
