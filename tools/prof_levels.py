"""Dev helper (GPU): per-launch device times of one LM trial at C2, aggregated by kernel and grid
size.  DEFTRI_PROFILE_DUMP makes deftri_profile_trial print every launch to stderr."""
import os, sys, pathlib, collections, subprocess
ROOT = pathlib.Path(__file__).resolve().parent.parent
if os.environ.get("DEFTRI_PROF_CHILD") is None:
    env = dict(os.environ, DEFTRI_PROF_CHILD="1")
    r = subprocess.run([sys.executable, __file__] + sys.argv[1:], env=env, capture_output=True, text=True)
    rows = [l.split() for l in r.stderr.splitlines() if l.startswith("[prof]")]
    print(r.stdout)
    if r.returncode:
        print(r.stderr[-3000:]); sys.exit(r.returncode)
    seq = [(n, int(g), float(ms)) for _, n, g, ms, _w, _l in rows]
    upd = [(int(g), float(ms), float(w)) for _, n, g, ms, w, _l in rows if n == "update"]
    lev = collections.defaultdict(lambda: collections.defaultdict(float))
    for _, n, g, ms, w, l in rows:
        lev[int(l)][n] += float(ms)
    with open(ROOT / "gpurun_out" / "prof_seq.txt", "w") as fo:
        for _, n, g, ms, w, l in rows:
            fo.write(f"{l} {n} {g} {1e3 * float(ms):.1f} {float(w) / 1e9:.4f}\n")
    print("per level (ms):")
    for l in sorted(lev):
        tot_l = sum(lev[l].values())
        print(f"  level {l:3d} total {tot_l:7.3f} " + " ".join(f"{k}={v:.3f}" for k, v in sorted(lev[l].items(), key=lambda kv: -kv[1])))
    print("update launches (grid, us, GF, TF/s), in order:")
    for i, (g, ms, w) in enumerate(upd):
        print(f"  {i:3d} grid {g:6d} {1e3 * ms:9.1f} us {w / 1e9:8.3f} GF {w / (ms * 1e-3) / 1e12:6.2f} TF/s")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, g, ms in seq:
        b = 1 if g <= 4 else 16 if g <= 64 else 256 if g <= 512 else 4096 if g <= 4096 else 10**9
        agg[(n, b)][0] += 1; agg[(n, b)][1] += ms
    tot = sum(ms for _, _, ms in seq)
    print(f"total device ms {tot:.3f} over {len(seq)} launches")
    for (n, b), (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:14s} grid<={b:<10d} launches {c:5d} ms {ms:8.3f} avg_us {1e3 * ms / c:8.2f}")
    sys.exit(0)
sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
import numpy as np
from deftri import capi, sim
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
m, _ = sim.simulate_two_view(n=n, seed=1, scale_scene=True, compact=True)
host = capi.Context(-1); p = host.build_graph(m, 1.0, 2e5, np.float32(0.003)); host.close()
ctx = capi.Context(0); ctx.upload(p)
ctx.profile_trial(1e3)
os.environ["DEFTRI_PROFILE_DUMP"] = "1"
st = ctx.profile_trial(1e3)
print({k: round(v["ms"], 3) for k, v in st.items()})
