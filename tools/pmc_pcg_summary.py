"""Summarize a tools/gpu_pmc_pcg.sh run into profiles/<tag>_pmc_pcg_product.json: HBM-side bytes of
k_pcg_product per active launch (FETCH_SIZE and WRITE_SIZE from separate rocprofv3 passes, KB*1024),
keyed by the plan's algorithmic bytes per launch so bench.py only attaches it to the same plan.

Launches past convergence return after the convergence test: only launches running longer than 30 %
of the longest are counted as active.  On gfx950 FETCH_SIZE reports 1/2 of the bytes of
16-byte-per-lane coalesced reads (MI355X_MICROARCH.md, HBM section); the product's slot records and
gathers are 16-byte loads, so the corrected fetch doubles the counter.

usage: python tools/pmc_pcg_summary.py gpurun_out/pmcpcg2 profiles/r02_pmc_pcg_product.json [kernel]
       (kernel: k_pcg_product, the default, or k_mf_product)
"""
import collections
import csv
import json
import pathlib
import sys


def per_dispatch(path, ctr, kernel):
    """per dispatch: (bytes, duration ns)"""
    vals = collections.defaultdict(float)
    dur = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != ctr or kernel not in r["Kernel_Name"]:
            continue
        vals[r["Dispatch_Id"]] += float(r["Counter_Value"]) * 1024.0
        dur[r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return vals, dur


def active(vals, dur):
    """launches that ran the product (not only the convergence test): duration above 30 % of the
    longest (the matrix-free product issues its first loads before the test, so bytes alone do not
    separate them)"""
    dmax = max(dur.values())
    return [v for k, v in vals.items() if dur[k] > 0.3 * dmax]


def main():
    src, dst = pathlib.Path(sys.argv[1]), pathlib.Path(sys.argv[2])
    k = sys.argv[3] if len(sys.argv) > 3 else "k_pcg_product"
    act_f = active(*per_dispatch(src / "fetch" / "run_counter_collection.csv", "FETCH_SIZE", k))
    act_w = active(*per_dispatch(src / "write" / "run_counter_collection.csv", "WRITE_SIZE", k))
    bench = json.loads((src / "fetch.json").read_text())
    alg = bench["roofline"]["bytes_per_launch"]
    fetch = sum(act_f) / len(act_f)
    write = sum(act_w) / len(act_w)
    out = {
        "kernel": k,
        "bytes_per_launch_algorithmic": alg,
        "active_launches": len(act_f),
        "fetch_bytes_per_launch_raw": fetch,
        "fetch_bytes_per_launch_corrected": 2.0 * fetch,
        "write_bytes_per_launch": write,
        "traffic_bytes_per_launch": 2.0 * fetch + write,
        "note": "rocprofv3 FETCH_SIZE / WRITE_SIZE in separate passes over `bench.py --steps 2 --warmup 1` "
                "(C2, PCG steps); active launches only; fetch corrected x2 for 16-byte lane loads (guide).",
    }
    dst.write_text(json.dumps(out, indent=1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
