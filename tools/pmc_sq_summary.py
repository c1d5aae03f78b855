"""Summary of the SQ counter passes of tools/r06_sq.sh: per tile-mode CG kernel (k_sp_tile, k_sp_tupd),
at C2 and 500k x 2, the per-dispatch means of every counter plus the derived shares — wave cycles parked
on memory / barriers (SQ_WAIT_ANY), issue-stalled (SQ_WAIT_INST_ANY), issuing (SQ_ACTIVE_INST_ANY) —
the mean wave lifetime (SQ_WAVE_CYCLES counts quad-cycles) and LDS bank-conflict cycles per LDS
instruction.  usage: python tools/pmc_sq_summary.py gpurun_out/r06sq > profiles/r06_sq_tile_kernels.json"""
import collections
import csv
import json
import pathlib
import sys

root = pathlib.Path(sys.argv[1])
out = {}
for corr in ("100000", "500000"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for g in ("g1", "g2"):
        f = root / f"c{corr}_{g}" / "run_counter_collection.csv"
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            name = "k_sp_tile" if "k_sp_tile" in k else "k_sp_tupd" if "k_sp_tupd" in k else None
            if name is None:
                continue
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[name] = {"vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]), "lds_bytes_static": int(r["LDS_Block_Size"]),
                          "workgroup": int(r["Workgroup_Size"]), "grid_threads": int(r["Grid_Size"])}
    res = {}
    for name, d in acc.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        wc = m["SQ_WAVE_CYCLES"]
        res[name] = dict(meta[name], dispatches=len(d["SQ_WAVES"]), counters={c: round(v, 1) for c, v in sorted(m.items())},
                         share_wait_any=round(m["SQ_WAIT_ANY"] / wc, 3), share_wait_inst=round(m["SQ_WAIT_INST_ANY"] / wc, 3),
                         share_active=round(m["SQ_ACTIVE_INST_ANY"] / wc, 3),
                         wave_lifetime_cycles=round(4 * wc / m["SQ_WAVES"]),
                         lds_conflict_cycles_per_lds_inst=round(m["SQ_LDS_BANK_CONFLICT"] / max(m["SQ_INSTS_LDS"], 1), 3))
    out["c2" if corr == "100000" else "500k_x2"] = res
print(json.dumps(out, indent=1))
