"""Summarize a tools/gpu_pmc.sh run into profiles/<tag>_pmc_k_update.json: k_update HBM bytes
(FETCH_SIZE + WRITE_SIZE, rocprofv3 reports KB) per factorization, keyed by the plan's update-flop
count so bench.py only attaches it to the same plan.

usage: python tools/pmc_summary.py gpurun_out/pmc1 profiles/r01_pmc_k_update.json
"""
import collections
import csv
import json
import sys
import pathlib


def load(path, ctr):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != ctr:
            continue
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("deftri::dev::", "").split("<")[0]
        agg[n][0] += 1
        agg[n][1] += float(r["Counter_Value"]) * 1024.0
    return agg


def main():
    src, dst = pathlib.Path(sys.argv[1]), pathlib.Path(sys.argv[2])
    f = load(src / "fetch" / "run_counter_collection.csv", "FETCH_SIZE")
    w = load(src / "write" / "run_counter_collection.csv", "WRITE_SIZE")
    bench = json.loads((src / "fetch.json").read_text())
    flops = bench["roofline"]["flops_per_factorization"]
    ndiag0 = f["k_diag"][0]
    # factorizations in the run = launches of k_update / launches per factorization (from the bench line)
    per_fact = bench["roofline"]["launches"]
    nfact = f["k_update"][0] / per_fact
    out = {
        "kernel": "k_update",
        "update_flops_per_factorization": flops,
        "factorizations_in_run": nfact,
        "fetch_bytes_per_factorization": f["k_update"][1] / nfact,
        "write_bytes_per_factorization": w["k_update"][1] / nfact,
        "note": "rocprofv3 FETCH_SIZE/WRITE_SIZE (separate passes), KB*1024, raw. k_update's operand panels "
                "are staged with 16-B/lane loads, for which the microarch guide measures FETCH_SIZE at 1/2 of "
                "the bytes: fetch_bytes_corrected doubles the fetch (an upper bound: the C-tile reads are "
                "8-B/lane)",
        "per_kernel_bytes_per_factorization": {k: {"fetch": f[k][1] / nfact, "write": w.get(k, [0, 0.0])[1] / nfact}
                                               for k in sorted(f, key=lambda k: -f[k][1])[:12]},
    }
    out["fetch_bytes_corrected_per_factorization"] = 2.0 * out["fetch_bytes_per_factorization"]
    out["traffic_bytes_per_factorization"] = (out["fetch_bytes_corrected_per_factorization"] +
                                              out["write_bytes_per_factorization"])
    dst.write_text(json.dumps(out, indent=1))
    print(json.dumps({k: out[k] for k in ("factorizations_in_run", "fetch_bytes_per_factorization",
                                          "write_bytes_per_factorization")}))


if __name__ == "__main__":
    main()
