"""Summarize tools/micro/fetch_calib under rocprofv3 (FETCH_SIZE and WRITE_SIZE passes) into the
measured counter / byte ratios per access width: profiles/<tag>_fetch_calibration.json.

usage: python tools/micro/fetch_calib_summary.py <fetch csv> <write csv> <out json>

Dispatches come in the program's order: per size (96 MiB, 768 MiB), 3 repetitions of
[read4, read8, read16, gather8, write8, write16].  Byte counts:
  read*   : the buffer (size bytes)
  gather8 : size / 2 of gathered doubles (each line of the first half read once) + size / 4 of int32 indices
  write*  : the buffer (size bytes)
The first repetition of the 96 MiB set comes from HBM; the next two can hit the Infinity Cache
(FETCH_SIZE counts its hits too: MI355X_MICROARCH.md §HBM)."""
import collections
import csv
import json
import sys

NAMES = ["read4", "read8", "read16", "gather8", "write8", "write16"]
SIZES = [96 << 20, 768 << 20]


def per_dispatch(path, ctr):
    """Per dispatch of the calibration kernels (the runtime's buffer fills in between are skipped)."""
    vals = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != ctr or not ("k_read" in r["Kernel_Name"] or "k_gather" in r["Kernel_Name"]
                                            or "k_write" in r["Kernel_Name"]):
            continue
        k = int(r["Dispatch_Id"])
        vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"]) * 1024.0
    return [vals[k] for k in sorted(vals)]


def expected(name, size):
    if name == "gather8":
        return size / 2 + size / 4
    return float(size)


def main():
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE")
    out = {"what": "rocprofv3 counter bytes / known bytes per dispatch, tools/micro/fetch_calib.hip", "cases": []}
    i = 0
    for size in SIZES:
        for rep in range(3):
            for name in NAMES:
                b = expected(name, size)
                f = fetch[i] if i < len(fetch) else None
                w = write[i] if i < len(write) else None
                out["cases"].append({"size": size, "rep": rep, "kernel": name, "bytes": b,
                                     "fetch_over_bytes": None if f is None else round(f / b, 4),
                                     "write_over_bytes": None if w is None else round(w / b, 4)})
                i += 1
    # the factors the CG kernels' PMC passes use: 768 MiB (past the Infinity Cache), last repetition
    big = {c["kernel"]: c for c in out["cases"] if c["size"] == SIZES[1] and c["rep"] == 2}
    out["factor_fetch_read8"] = big["read8"]["fetch_over_bytes"]
    out["factor_fetch_read16"] = big["read16"]["fetch_over_bytes"]
    out["factor_fetch_read4"] = big["read4"]["fetch_over_bytes"]
    out["factor_fetch_gather8"] = big["gather8"]["fetch_over_bytes"]
    out["factor_write8"] = big["write8"]["write_over_bytes"]
    out["factor_write16"] = big["write16"]["write_over_bytes"]
    with open(sys.argv[3], "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k.startswith("factor")}, indent=1))
    for c in out["cases"]:
        if c["rep"] == 2:
            print(c)


if __name__ == "__main__":
    main()
