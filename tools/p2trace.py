"""Summarize a phase-2 wave trace (DEFTRI_SP_P2_TRACE=<file>, spcg.hip k_sp_phase2 stamps): per wave
[start, rows / heavy sums done, alpha known, end, hw id, slot steps] on the 100 MHz wall clock.

usage: python tools/p2trace.py <trace file> [json out]
Prints the launch span, start-time spread (waves that wait for a free slot start late), and the
quantiles of each stage's duration."""
import json
import sys

import numpy as np


def main():
    raw = np.fromfile(sys.argv[1], dtype=np.int64)
    nw, m_nh, rs, p2u = (int(v) for v in raw[:4])
    t = raw[4:].reshape(-1, 6)[:nw]
    live = t[:, 0] > 0
    t = t[live]
    ids = np.nonzero(live)[0]
    t0 = t[:, 0].min()
    us = 0.01                                            # 100 MHz: 10 ns per tick
    start, rows, alpha, end = ((t[:, i] - t0) * us for i in range(4))
    hw = t[:, 4]
    heavy = ids // 4 < m_nh
    q = [0, 10, 50, 90, 99, 100]

    def qs(a):
        return [round(float(v), 2) for v in np.percentile(a, q)] if a.size else []

    r = ~heavy
    out = {
        "waves": int(t.shape[0]), "heavy_waves": int(heavy.sum()), "rs": rs, "p2u": p2u,
        "span_us": round(float(end.max()), 2),
        "quantiles": q,
        "start_us": qs(start[r]),
        "slot_loop_us": qs((rows - start)[r]),
        "alpha_wait_us": qs((alpha - rows)[r]),
        "tail_us (update + tickets)": qs((end - alpha)[r]),
        "wave_life_us": qs((end - start)[r]),
        "end_us": qs(end[r]),
        "steps": qs(t[r, 5].astype(float)),
        "heavy_end_us": qs(end[heavy]),
        "alpha_known_first_us": round(float(alpha[r].min()), 2) if r.any() else None,
        "late_starts (start > 2 us)": int((start[r] > 2.0).sum()),
        "distinct_hw_ids": int(np.unique(hw).size),
    }
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
