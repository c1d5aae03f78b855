"""Timeline of a rocprofv3 --kernel-trace run: per kernel name the launches, busy time and the idle
gap before each launch (device idle between the previous kernel's end and this one's start), and
over the whole trace the busy fraction — what the timed loop spends outside kernels (host round
trips, launch latency, dependency gaps).

usage: python tools/trace_gaps.py KERNEL_TRACE.csv [--window NAME] [--json OUT]
  --window: the launches strictly between the first and the last kernel whose name contains NAME
            (bench.py --trace-markers brackets the timed region with a torch MulFunctor kernel)
"""
import argparse
import collections
import csv
import glob
import os
import json
import re


def short(name):
    m = re.search(r"(k_[A-Za-z0-9_]+)", name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--window")
    ap.add_argument("--json")
    a = ap.parse_args()
    path = a.csv
    if os.path.isdir(path):          # a rocprofv3 output directory: its kernel trace
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    if a.window:
        idx = [i for i, e in enumerate(ev) if a.window in e[2]]
        ev = ev[idx[0] + 1:idx[-1]]
    ev = [(s, e, short(n)) for s, e, n in ev]
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    busy = collections.defaultdict(float)
    gaps = collections.defaultdict(float)
    cnt = collections.Counter()
    prev_end = ev[0][0]
    for s, e, n in ev:
        cnt[n] += 1
        busy[n] += (e - s) * 1e-3
        gaps[n] += max(0, s - prev_end) * 1e-3
        prev_end = max(prev_end, e)
    wall = (t1 - t0) * 1e-3
    tot_busy = sum(busy.values())
    tot_gap = sum(gaps.values())
    out = {"wall_us": round(wall, 1), "busy_us": round(tot_busy, 1), "gap_us": round(tot_gap, 1),
           "busy_frac": round(tot_busy / wall, 4), "launches": sum(cnt.values()),
           "kernels": {n: {"launches": cnt[n], "busy_us": round(busy[n], 1), "avg_us": round(busy[n] / cnt[n], 2),
                           "gap_before_us": round(gaps[n], 1), "avg_gap_us": round(gaps[n] / cnt[n], 2)}
                       for n in sorted(busy, key=lambda k: -busy[k] - gaps[k])}}
    print(f"wall {wall:.0f} us, kernels busy {tot_busy:.0f} us ({100 * tot_busy / wall:.1f} %), idle gaps {tot_gap:.0f} us, "
          f"{out['launches']} launches")
    print(f"{'kernel':28s} {'n':>6s} {'busy us':>10s} {'avg':>8s} {'gap us':>10s} {'avg gap':>8s}")
    for n, k in out["kernels"].items():
        print(f"{n:28s} {k['launches']:6d} {k['busy_us']:10.1f} {k['avg_us']:8.2f} {k['gap_before_us']:10.1f} {k['avg_gap_us']:8.2f}")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
