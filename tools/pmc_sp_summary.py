"""Summarize a tools/archive/r03_prof.sh run into profiles/<tag>_pmc_sp_product.json: HBM-side bytes of the
iterative plan's CG iteration (k_sp_tile + k_sp_tupd in tile mode, k_sp_phase1 + k_sp_phase2 otherwise)
per active launch pair, from rocprofv3 FETCH_SIZE and WRITE_SIZE passes (separate runs, KB * 1024), keyed by the plan's
algorithmic bytes per product so bench.py attaches it only to the same plan.

Launches past convergence return after the state test: only launches longer than 30 % of the
kernel's longest are counted as active.  FETCH_SIZE is reported raw: the guide calibrates it at 1/2
for 16-byte-per-lane coalesced reads; these kernels read 8-byte lanes (column-major J, packed slots)
and 16-byte (z, p) gathers, an uncalibrated mix — `fetch_bytes_x2` gives the upper bound.

usage: python tools/pmc_sp_summary.py gpurun_out/<tag> profiles/<tag>_pmc_sp_product.json [WORKLOAD]
"""
import collections
import csv
import json
import pathlib
import sys


def per_dispatch(path, ctr, kernel):
    vals = collections.defaultdict(float)
    dur = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != ctr or kernel not in r["Kernel_Name"]:
            continue
        vals[r["Dispatch_Id"]] += float(r["Counter_Value"]) * 1024.0
        dur[r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return vals, dur


def active_mean(vals, dur):
    dmax = max(dur.values())
    act = [(v, dur[k]) for k, v in vals.items() if dur[k] > 0.3 * dmax]
    return sum(v for v, _ in act) / len(act), sum(d for _, d in act) / len(act), len(act)


def main():
    src, dst = pathlib.Path(sys.argv[1]), pathlib.Path(sys.argv[2])
    wl = sys.argv[3] if len(sys.argv) > 3 else "C2"
    bench = json.loads((src / "pmc_fetch.json").read_text())
    alg = bench["roofline"]["bytes_per_launch"]
    names = [bench["roofline"]["phase1"].get("kernel", "k_sp_phase1"), bench["roofline"]["phase2"].get("kernel", "k_sp_phase2")]
    fcsv = (src / "fetch" / "run_counter_collection.csv").read_text()
    names = [k for k in names if k + "<" in fcsv or k + "(" in fcsv]        # (the fused tile chain: one kernel)
    out = {"kernel": "+".join(names), "bytes_per_launch_algorithmic": alg, "per_kernel": {}}
    tf = tw = 0.0
    for k in names:
        f, df, nf = active_mean(*per_dispatch(src / "fetch" / "run_counter_collection.csv", "FETCH_SIZE", k))
        w, dw, nw = active_mean(*per_dispatch(src / "write" / "run_counter_collection.csv", "WRITE_SIZE", k))
        out["per_kernel"][k] = {"fetch_bytes_raw": f, "write_bytes": w, "active_launches": nf, "mean_ns": df}
        tf += f
        tw += w
    out.update({"fetch_bytes_per_launch_raw": tf, "fetch_bytes_x2": 2 * tf, "write_bytes_per_launch": tw,
                "traffic_bytes_per_launch": tf + tw,
                "traffic_over_algorithmic": (tf + tw) / alg,
                "note": "rocprofv3 FETCH_SIZE / WRITE_SIZE in separate passes over `bench.py --steps 3 --warmup 1 "
                        f"--no-cpu-baseline --no-e2e` ({wl}, iterative plan); active launches only; FETCH_SIZE raw "
                        "(8-B lane reads: uncalibrated; x2 = the 16-B-lane calibration, an upper bound)"})
    dst.write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
