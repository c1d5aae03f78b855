"""Headline benchmark: LM iterations/s of the g2o ARAP solve (arapOptimization's
optimizer.optimize(nIterations), reference Modules/Optimization/g2oBundleAdjustment.cc:959-962) at
config C2 of BASELINE.json: 100k two-view correspondences.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--corr 100000] [--no-cpu-baseline]
                  [--analytic] [--solver pcg|direct] [--sharded] [--cpu-full-iteration]
  python bench.py --workload ba [--ba-points 500000] [--ba-kfs 8] [--ba-scaling strong|weak] ...

A "step" is one LM iteration of the device solver (linearize with g2o's numeric ARAP/depth
Jacobians — the reference's arithmetic — assemble H, then up to 10 damped trials, each a step
solve (block-Jacobi PCG, or the multifrontal LDL^T) + update + chi2).  The scene is synthetic (deftri.sim: the
reference's simulation recipe scaled to n points); the graph is built on the host once, then
resident in HBM before the timed region starts.

Multi-GPU (N > 1, one process per GPU, RCCL): the BASELINE metric's fixed problem (C2, 100k
correspondences x 2 views) point-sharded over the N ranks — strong scaling, value = that problem's
LM iterations/s.  The iterative plan (csrc/spcg.h): each rank owns a contiguous Morton range of point
rows; per CG iteration one ncclAllReduce of [r.z, r.r, z.Az, the global vertices' sums] and one
grouped send / receive of the boundary rows, overlapped with the interior edges' product
(DESIGN.md §7).  The line also carries `north_star_500k`: the 500k x 2 problem (3M unknowns, the
north star's size) split the same way.  --weak: one problem of N x 100k correspondences instead
(value in C2-equivalent iterations/s).  --replicas: N independent C2 problems (no collective;
per-problem rate).  --solver direct runs the sharded multifrontal LDL^T instead.  The barrier and the
max-over-ranks time use torch.distributed.

Legs of the default C2 line (--no-legs skips them): `north_star_500k` (above, any N); at N > 1 `c4`:
BASELINE C4 (8 keyframes x 500k, all 28 pairs, 12M unknowns) point-sharded over the same ranks, 1 +
min(steps, 3) LM iterations (strong scaling; the multi-pair graph's sharded chain); and, at N = 1,
`regimes.realcolon`: the C2 scene under Realcolon.yaml's weights and camera (arap 0.1, sigma_d 1e-6 m,
KB8 d0..d3; Data/Realcolon.yaml:15-23,101,110), a CG-heavy regime (the Simulation.yaml headline
run is near-stalled: ~5 CG iterations per trial at lambda ~1e21).

Printed roofline (the iterative plan, the default): the CG iteration's kernels — at C2 (one rank, one
pair: tile mode) k_sp_tile (the matrix-free product, every ARAP edge read once) + k_sp_tupd (the
update); otherwise k_sp_phase1 + k_sp_phase2 (the product with the update folded in) — HBM-bound, from a profiled trial
right after the timed region (HIP events on the solver's own stream, active launches only).  Two
fractions of 8 TB/s: `frac` / `frac_survey` on SURVEY.md §8(d)'s minimal-traffic bytes per CG
iteration (176 E + 48 R + 40 D + 156 P: fp32 Jacobians, one pass over the edges), and `frac_design`
on the bytes this design actually moves (fp64 J stored column-major for phase 1 and again per slot
for phase 2, the s_e round trip, the (z, p) pairs: the plan's own count).  `traffic` from the
committed rocprofv3 PMC pass when it matches the plan, with the calibrated FETCH_SIZE factor
(profiles/*_fetch_calibration.json) and `traffic_over_survey_bytes`.

A "step" is one LM iteration; with PCG steps each trial is setup + CG iterations (product, heavy
rows, update) instead of scatter + factorization + substitution.

CPU baseline: the oracle (oracle/deftri_oracle.c: the reference LM restated in scalar C, g2o
numeric Jacobians, SimplicialLDLT) on the SAME full-size C2 problem with the device plan's
elimination order, 1 thread: one linearization and one trial are measured; the per-iteration
figure is linearization + (GPU trials per iteration) x trial.  --cpu-full-iteration times a
complete first LM iteration instead.
"""
import argparse
import json
import os
import pathlib
import sys
import time

# torch first: libdeftri then binds to the HIP runtime torch already loaded (same soname), so
# torch.cuda.synchronize() and the solver share one runtime.
import torch
import torch.distributed as dist

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
import numpy as np  # noqa: E402

from deftri import capi, sim  # noqa: E402

FP64_PEAK_TFLOPS = 78.6
HBM_PEAK_GBS = 8000.0              # MI355X HBM3E spec (MI355X_MICROARCH.md; 6.29 TB/s measured copy)
MFMA_F64_SUSTAINED_TFLOPS = 48.3   # v_mfma_f64_16x16x4 back-to-back on this box (tools/micro/mfma_f64_peak.hip)
BASELINE_METRIC = "LM iterations/sec + ms/iter at 100k corr \u00d7 2 views; 1/2/4/8-GPU scaling"
REP_W, ARAP_W, DEPTH_SIGMA = 1.0, 2e5, np.float32(3.0 / 1000.0)
# the C2 scene under the three weight regimes of the reference's data sets (rep, arap, sigma_d, KB8):
# Simulation.yaml; Drunkard.yaml:68,77 (DepthWeight 0.3 mm); Realcolon.yaml:15-23,101,110 (DepthWeight
# 0.001 -> 1e-6 m, information 1e12, arap 0.1, distorted KB8)
REGIME = "simulation"
REGIMES = {
    "simulation": (1.0, 2e5, np.float32(3.0 / 1000.0), None),
    "drunkard": (1.0, 1e7, np.float32(0.3) / np.float32(1000.0), "DRUNKARD_KB8"),
    "realcolon": (1.0, 0.1, np.float32(0.001) / np.float32(1000.0), "REALCOLON_KB8"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_problem(n, seed, regime="simulation"):
    rep, arap, sig, kb8 = REGIMES[regime]
    return sim.two_view_problem(n, seed, rep, arap, sig, return_map=True,
                                kb8=getattr(sim, kb8) if kb8 else None)


def end_to_end(device, m, configure, n_it=25):
    """The drop-in call a caller of the reference's arapOptimization makes (g2oBundleAdjustment.cc:608,
    Simulation.yaml weights rep 1 / global 50 / arap 2e5, nIt 25): host graph build + upload + device
    LM + write-back.  `*_call_s` brackets the C-ABI call alone (what a C++ caller pays); `*_s` adds
    this Python harness's map marshalling.  Three calls:
      cold        a fresh context (graph build, plan build, first-touch allocations)
      warm        the same context, a clone of the same map: NLopt's outerObjective evaluations
                  (nloptOptimization.cc:4-37) — the graph memo and the plan are reused
      next_round  the same context, the map the warm call wrote back: deformationOptimization's
                  next round — positions moved, so the graph and the plan are built again"""
    import copy
    out = {"n_iterations": n_it}
    fresh = capi.Context(device)
    configure(fresh)
    mm = None
    for key, c, src in (("cold", fresh, m), ("warm", fresh, m), ("next_round", fresh, None)):
        mm = copy.deepcopy(src) if src is not None else mm
        t0 = time.perf_counter()
        _, rep = c.arap_optimization(mm, REP_W, 50.0, ARAP_W, 1.0, 1.0, DEPTH_SIGMA, n_it)
        out[key + "_s"] = round(time.perf_counter() - t0, 3)
        out[key + "_call_s"] = round(c.last_call_s, 4)
        out[key + "_lm_s"] = round(rep["ms_total"] * 1e-3, 4)
        out[key + "_iterations"] = rep["iterations"]
        out[key + "_plan_reuses"] = rep["plan_reuses"]
        mh, sh, gms = c.graph_stats()
        nrep, nfl = c.graph_repairs()
        out[key + "_graph_ms"] = round(gms, 2)
        out[key + "_graph_path"] = "memo" if mh > out.get("_mh", 0) else ("structure memo" if sh > out.get("_sh", 0) else "full")
        if out[key + "_graph_path"] == "full" and nrep > out.get("_rep", 0):
            out[key + "_graph_path"] = f"full (mesh flip-repaired: {nfl - out.get('_fl', 0)} flips)"
        out["_mh"], out["_sh"], out["_rep"], out["_fl"] = mh, sh, nrep, nfl
    fresh.close()
    for k in ("_mh", "_sh", "_rep", "_fl"):
        out.pop(k, None)
    return out


def host_cpu_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "cpu_model": model}


def cpu_baseline(prob, order, gpu_trials_per_iter, full_iteration=False):
    """The oracle (scalar C, 1 thread) on the benchmark's own full-size problem, eliminating in the
    device plan's order.  Measured: one linearization + one LM trial (or, with full_iteration, the
    first LM iteration with all its trials)."""
    sys.path.insert(0, str(ROOT))
    from oracle import oracle
    import threading
    oracle.set_vertex_order(order)
    t = time.perf_counter()
    done = threading.Event()

    def heartbeat():                 # the oracle call is one long C call (ctypes drops the GIL)
        while not done.wait(30.0):
            log(f"cpu baseline: oracle running, {time.perf_counter() - t:.0f} s")
    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()
    try:
        r = oracle.solve_lm(prob, 1, analytic=False, max_trials=10 if full_iteration else 1)["report"]
    finally:
        done.set()
    dt = time.perf_counter() - t
    oracle.set_vertex_order(None)
    trials = max(r["trials_total"], 1)
    lin = r["ms_linearize"] * 1e-3
    per_trial = (r["ms_factor"] + r["ms_solve"] + r["ms_update"]) * 1e-3 / trials
    if full_iteration:
        t_iter, how = dt, f"first LM iteration measured whole ({trials} trials, {dt:.1f} s)"
    else:
        t_iter = lin + gpu_trials_per_iter * per_trial
        how = (f"measured: linearization {lin:.2f} s + one trial {per_trial:.2f} s (factor + solve + update + chi2); "
               f"per iteration = linearization + {gpu_trials_per_iter:.2f} trials (the GPU's trials per iteration)")
    info = host_cpu_info()
    return {"value": 1.0 / t_iter, "unit": "LM iterations/s", "cores": 1, "kind": "port",
            "sample": f"oracle LM (g2o numeric J, SimplicialLDLT in the device plan's elimination order) on the full "
                      f"{prob.n_points // 2}-correspondence x 2-view problem, 1 thread; {how}; "
                      f"host {info['cpu_model']}, nproc {info['nproc']}",
            "seconds_per_iteration": round(t_iter, 3), "seconds_per_trial": round(per_trial, 3),
            "seconds_linearize": round(lin, 3), "nproc": info["nproc"], "cpu_model": info["cpu_model"]}


def ba_cpu_baseline(prob, n_iter=3):
    """The BA oracle (oracle/ba_oracle.c: g2o BlockSolver_6_3 Schur LM restated in C, 1 thread) on
    the benchmark's own scene (rank 0's shard = the whole scene at N=1): n_iter LM iterations
    timed, nothing extrapolated."""
    sys.path.insert(0, str(ROOT))
    from oracle import oracle
    t = time.perf_counter()
    r = oracle.ba_solve(prob, n_iter)["report"]
    dt = time.perf_counter() - t
    it = max(r["iterations"], 1)
    return {"value": it / dt, "unit": "LM iterations/s", "cores": 1, "kind": "port",
            "sample": f"BA oracle LM on the same {prob.n_points}-point x {prob.n_poses}-KF scene ({prob.n_edges} edges): "
                      f"{r['iterations']} iterations ({r['trials_total']} trials) in {dt:.2f} s"}


def main_ba(args, world, rank, gpu, backend):
    """Point-sharded bundle adjustment (SURVEY §8 a14 / e): the BlockSolver_6_3 Schur LM on every
    rank's point shard, RCCL all-reduce of the pose blocks and the Schur complement per LM trial.
    strong: the --ba-points scene split over the ranks; weak: --ba-points per rank."""
    from deftri import ba
    n_total = args.ba_points if args.ba_scaling == "strong" else args.ba_points * world
    t0 = time.perf_counter()
    full = ba.make_ba_problem(n=n_total, k=args.ba_kfs, seed=1, outliers=0.01)
    prob, (lo, hi), _ = full.shard(rank, world)
    log(f"[rank {rank}] BA scene {full.n_points} points x {full.n_poses} KFs, {full.n_edges} edges; shard "
        f"[{lo}, {hi}) with {prob.n_edges} edges, built in {time.perf_counter() - t0:.1f}s")
    ctx = capi.BAContext(gpu)
    if world > 1:
        if backend == "nccl":
            uid = [capi.rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            ctx.dist_init_rccl(world, rank, uid[0])
        else:
            def allreduce(buf, op):
                t = torch.from_numpy(buf)
                dist.all_reduce(t, op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MAX)
            ctx.dist_set_allreduce(world, rank, allreduce)
    ctx.upload(prob)
    if args.warmup > 0:
        ctx.solve_lm(args.warmup)
    ctx.set_state(poses=prob.poses, points=prob.points)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rep = ctx.solve_lm(args.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    log(f"[rank {rank}] BA {rep['iterations']} iterations / {rep['trials_total']} trials in {dt * 1e3:.1f} ms; "
        f"chi2 {rep['chi2_initial']:.6e} -> {rep['chi2_final']:.6e}")
    iters = rep["iterations"]
    t_max, _, _ = reduce_stats(dt, iters, rep["trials_total"], world, "cuda" if backend == "nccl" else "cpu")
    value = iters / t_max
    stats = ctx.profile_trial(rep["lambda_final"])
    # roofline: the edge linearization kernel (the dominant HBM stream): algorithmic bytes of one
    # trial's two ba_edges launches / their device time
    ed = stats.get("ba_edges", {"ms": 0.0, "bytes": 0.0, "launches": 0})
    achieved = ed["bytes"] / max(ed["ms"] * 1e-3, 1e-12) / 1e9
    roofline = {"bound": "hbm", "kernel": "ba_edges", "achieved": round(achieved, 1), "peak": 8000.0,
                "unit": "GB/s", "frac": round(achieved / 8000.0, 4), "traffic": None,
                "bytes_per_trial": ed["bytes"], "launches": ed["launches"],
                "avg_launch_us": round(1e3 * ed["ms"] / max(ed["launches"], 1), 3)}
    trial_ms = {k: round(v["ms"], 4) for k, v in sorted(stats.items(), key=lambda kv: -kv[1]["ms"])}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = ba_cpu_baseline(prob)
        log(f"BA cpu baseline: {cpu}")
    if rank == 0:
        out = {
            "metric": "BA LM iterations/sec (BlockSolver_6_3 Schur, point-sharded)",
            "value": value, "unit": "LM iterations/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * t_max / max(iters, 1), "higher_is_better": True,
            "scaling": args.ba_scaling, "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"BA-{full.n_points // 1000}k-x{full.n_poses}", "points": full.n_points,
                       "keyframes": full.n_poses, "edges": full.n_edges, "points_per_gpu": hi - lo,
                       "free_pose_dofs": 6 * (full.n_poses - 1),
                       "trials_per_iteration": round(rep["trials_total"] / max(iters, 1), 3),
                       "parallelism": f"points{world}"},
            "roofline": roofline, "cpu_baseline": cpu, "trial_kernel_ms": trial_ms,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def main_deformation(args, world, rank, gpu):
    """deformationOptimization end to end (g2oBundleAdjustment.cc:446-606) at the Simulation.yaml
    defaults (tests/golden/sim_default/settings.yaml is Data/Simulation.yaml byte for byte: 20 outer
    rounds, twoOptimizations + nlopt with 30 Nelder-Mead evaluations per round — every evaluation an
    arapOptimization of 25 LM iterations on a map clone (outerObjective, nloptOptimization.cc:4-37) —
    then arapOptimization with the optimum; stop at sum |dp| < 1e-4 |MapPoints|; the documented
    DepthWeight deviation 3.0) on the reference's simulation scene scaled to --corr
    correspondences (C1: 1000).  Times the whole call on the device; the CPU leg runs the same loop
    with the oracle's arapOptimization (tests/arap_oracle_fn.py: oracle/graph_ref.py graph build +
    the oracle LM, 1 thread) for its first outer round (a bounded sample), compared round for round."""
    import copy
    from deftri import optimization
    from deftri.settings import Settings
    n = args.corr or 1000
    st = Settings(path=str(ROOT / "tests" / "golden" / "sim_default" / "settings.yaml"))
    st.depth_weight = 3.0
    if args.rounds:
        st.n_optimizations = args.rounds
    m, _ = sim.simulate_two_view(n=n, seed=1, scale_scene=True, compact=True)
    m0 = copy.deepcopy(m)
    rounds = []
    t0 = time.perf_counter()
    t_last = [t0]

    def log_round(info):
        t = time.perf_counter()
        rounds.append({"round": info["round"], "s": round(t - t_last[0], 3), "evaluations": len(info.get("evaluations", [])),
                       "weights": info.get("weights"), "update": info["update"]})
        t_last[0] = t
    out_rounds = optimization.deformationOptimization(m, st, device=gpu, log=log_round)
    dt = time.perf_counter() - t0
    n_eval = sum(len(r.get("evaluations", [])) + 1 for r in out_rounds)
    log(f"deformation: {len(out_rounds)} rounds, {n_eval} arapOptimization calls in {dt:.2f} s")
    cpu = None
    if not args.no_cpu_baseline:
        # one arapOptimization of the loop (the first Nelder-Mead evaluation: the map's clone at the
        # Simulation.yaml weights, 25 LM iterations) on the oracle — ~13 s of one core at 1k; the
        # whole first round (8 calls) is ~100 s
        sys.path.insert(0, str(ROOT))
        sys.path.insert(0, str(ROOT / "tests"))
        from arap_oracle_fn import oracle_arap
        mc = copy.deepcopy(m0)
        t1 = time.perf_counter()
        upd = oracle_arap(mc, st.rep, st.global_, st.arap, st.alpha, st.beta, st.depth_sigma, st.n_iterations)
        dc = time.perf_counter() - t1
        info = host_cpu_info()
        cpu = {"value": 1.0 / dc, "unit": "arapOptimization calls/s", "cores": 1, "kind": "port",
               "sample": f"one arapOptimization of the loop (a clone of the {n}-correspondence map at the Simulation.yaml "
                         f"weights, {st.n_iterations} LM iterations) with the oracle (Python graph build + C LM, 1 thread): "
                         f"{dc:.2f} s, update {upd:.6g}; host {info['cpu_model']}",
               "seconds_per_call": round(dc, 3)}
        log(f"deformation cpu baseline: {cpu}")
    out = {"metric": "arapOptimization calls/s inside deformationOptimization (Simulation.yaml defaults, NLopt weight search)",
           "value": n_eval / dt, "unit": "arapOptimization calls/s", "n_gpus": 1, "steps": n_eval,
           "warmup": 0, "ms_per_step": 1e3 * dt / max(n_eval, 1), "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": f"deformation-{n}", "correspondences": n, "rounds": len(out_rounds),
                      "arap_calls": n_eval, "seconds_total": round(dt, 3), "outer_rounds_per_s": round(len(out_rounds) / dt, 4),
                      "settings": "Data/Simulation.yaml (+ DepthWeight 3.0)"},
           "rounds": rounds, "roofline": None, "cpu_baseline": cpu}
    print(json.dumps(out), flush=True)


def reduce_stats(dt, iters, trials, world, device):
    """Whole-job numbers from per-rank ones: max wall time over ranks, summed iterations/trials.
    The replicas share nothing else (no data-path collective)."""
    if world <= 1:
        return dt, iters, trials
    v = torch.tensor([dt], dtype=torch.float64, device=device)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    s = torch.tensor([iters, trials], dtype=torch.float64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    return float(v.item()), int(s[0].item()), int(s[1].item())


def job_rate(t_max, iters, units=1):
    """value and ms/step of the ARAP bench line: the LM iterations of ONE problem over the slowest
    rank's wall time — sharded, every rank ran the same iterations of the one problem; replicas, each
    rank its own copy, so the rate is per problem (never a sum over ranks).  units: the workload-sized
    shares one iteration of the problem covers (weak scaling: N, each rank holding one share), so
    value counts the correspondence-iterations of all ranks in units of the N = 1 iteration."""
    return iters * units / t_max, 1e3 * t_max / max(iters, 1)


# BASELINE workloads of the ARAP LM: scene recipe, weights (rep, arap, depth sigma) and
# keyframe-pair window; --corr overrides the correspondences per keyframe
WORKLOADS = {
    "c2": {"k": 2, "n": 100000, "desc": "two-view deformable triangulation (Simulation.yaml weights)"},
    "c3": {"k": 8, "n": 50000, "kb8": "drunkard", "w": (1.0, 1e7, 0.3), "window": 0,
           "desc": "8 keyframes x 50k, all 28 pairs (Drunkard.yaml shapes / weights)"},
    "c4": {"k": 8, "n": 500000, "kb8": "drunkard", "w": (1.0, 1e7, 0.3), "window": 0,
           "desc": "500k map points per keyframe x 8 keyframes, all 28 pairs (Drunkard.yaml shapes / weights)"},
    "c5": {"k": 20, "n": 200000, "kb8": "realcolon", "w": (1.0, 0.1, 1e-6), "window": 1,
           "desc": "Realcolon.yaml: 20 keyframes x 200k, DepthWeight 0.001 (info 1e12), arap 0.1"},
}


def build_workload(wl, n, seed, window):
    spec = WORKLOADS[wl]
    if wl == "c2":
        prob, m = build_problem(n, seed, REGIME)
        return prob, m
    kb8 = sim.DRUNKARD_KB8 if spec["kb8"] == "drunkard" else sim.REALCOLON_KB8
    rep, arap, sig = spec["w"]
    return sim.multi_view_problem(n, spec["k"], seed=seed, kb8=kb8, rep_weight=rep, arap_weight=arap,
                                  depth_sigma=np.float32(sig), pair_window=window), None


def cpu_baseline_sample(wl, window, n_sample, gpu_trials_per_iter):
    """The oracle (1 thread) on a bounded sample of a multi-keyframe workload: the same recipe at
    n_sample correspondences per keyframe (the full C3-C5 sizes take hours in scalar SimplicialLDLT);
    one linearization + one trial measured, per iteration = linearization + the GPU's trials per
    iteration x trial."""
    sys.path.insert(0, str(ROOT))
    from oracle import oracle
    import threading
    prob, _ = build_workload(wl, n_sample, 1, window)
    with capi.Context(-1) as hc:          # eliminate in the host analysis's order, as for C2
        hc.analyse(prob)
        oracle.set_vertex_order(hc.vertex_order())
    t = time.perf_counter()
    done = threading.Event()

    def heartbeat():
        while not done.wait(30.0):
            log(f"cpu baseline ({wl} sample): oracle running, {time.perf_counter() - t:.0f} s")
    threading.Thread(target=heartbeat, daemon=True).start()
    try:
        r = oracle.solve_lm(prob, 1, analytic=False, max_trials=1)["report"]
    finally:
        done.set()
        oracle.set_vertex_order(None)
    dt = time.perf_counter() - t
    lin = r["ms_linearize"] * 1e-3
    per_trial = (r["ms_factor"] + r["ms_solve"] + r["ms_update"]) * 1e-3 / max(r["trials_total"], 1)
    t_iter = lin + gpu_trials_per_iter * per_trial
    info = host_cpu_info()
    return {"value": 1.0 / t_iter, "unit": "LM iterations/s", "cores": 1, "kind": "port",
            "sample": f"oracle LM (g2o numeric J, SimplicialLDLT in the host analysis's elimination order) on the {wl} recipe at {n_sample} correspondences per "
                      f"keyframe ({prob.n_unknowns} unknowns, {len(prob.arap_pair)} ARAP edges), 1 thread: linearization "
                      f"{lin:.2f} s + one trial {per_trial:.2f} s, per iteration = linearization + "
                      f"{gpu_trials_per_iter:.2f} trials; {dt:.1f} s measured; host {info['cpu_model']}",
            "seconds_per_iteration": round(t_iter, 3), "sample_unknowns": prob.n_unknowns}


def fetch_calibration():
    """The committed FETCH_SIZE calibration of the access widths the CG kernels use
    (tools/micro/fetch_calib.hip under rocprofv3, profiles/*_fetch_calibration.json), or None."""
    for pm in sorted(ROOT.glob("profiles/*_fetch_calibration.json"), reverse=True):
        return json.loads(pm.read_text()), pm.name
    return None, None


def product_roofline(stats, rep, ctx, rank):
    """Roofline of the step solver's dominant kernel from a profiled trial (HIP events on the solver
    stream): active launches only (the profiled replay launches exactly the solve's CG iterations)."""
    tile = "sp_tile" in stats
    if tile or "sp_phase1" in stats:
        # tile mode (one rank: one pair or several): k_sp_tile (the product, every ARAP edge read once)
        # + k_sp_tupd (the update) (the sharded tile chain: k_sp_tile (interior + boundary launches) +
        # k_sp_update_sd)
        n1, n2 = ("sp_tile", "sp_tupd" if "sp_tupd" in stats else "sp_update") if tile else ("sp_phase1", "sp_phase2")
        none = {"launches": 0, "ms": 0.0, "bytes": 0.0}
        p1, p2 = stats[n1], stats.get(n2, none)
        its = max(p2["launches"] or p1["launches"], 1)
        by, ms = p1["bytes"] + p2["bytes"], p1["ms"] + p2["ms"]
        gbs = by / max(ms * 1e-3, 1e-12) / 1e9
        survey = ctx.plan_info().get("survey_bytes") or 0.0
        gbs_s = survey / max(ms / its * 1e-3, 1e-12) / 1e9
        cg = sum(stats[k]["ms"] for k in ("sp_dots", "sp_phase1", "sp_phase2", "sp_heavy", "sp_update", "sp_tile",
                                          "sp_tupd", "sp_alpha", "sp_txb") if k in stats)
        merged = "sp_update" not in stats
        if tile and n2 == "sp_update":
            kname = "k_sp_tile+k_sp_update_sd (sharded tile chain: A z by tiles, every ARAP edge read once + update)"
        elif tile:
            kname = "k_sp_tile+k_sp_tupd (tile mode: matrix-free product reading every ARAP edge once + update)"
        else:
            kname = ("k_sp_phase1+k_sp_phase2 (merged CG iteration: matrix-free product + p.Ap row terms + update)"
                     if merged else "k_sp_phase1+k_sp_phase2 (matrix-free product)")
        out = {"bound": "hbm", "kernel": kname, "achieved": round(gbs_s, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs_s / HBM_PEAK_GBS, 4), "traffic": None,
                "bytes_basis": "SURVEY.md 8(d) B_pcg = 176E + 48R + 40D + 156P per CG iteration",
                "survey_bytes_per_cg_iteration": survey,
                "frac_survey": round(gbs_s / HBM_PEAK_GBS, 4),
                "achieved_design": round(gbs, 1), "frac_design": round(gbs / HBM_PEAK_GBS, 4),
                "traffic_unit": "bytes per product", "bytes_per_launch": by / its, "launches": its,
                "avg_active_launch_us": round(1e3 * ms / its, 3),
                "phase1": {"kernel": "k_" + n1, "us": round(1e3 * p1["ms"] / its, 3), "bytes": p1["bytes"] / its,
                           "gbs": round(p1["bytes"] / max(p1["ms"] * 1e-3, 1e-12) / 1e9, 1)},
                "phase2": {"kernel": "k_" + n2, "us": round(1e3 * p2["ms"] / its, 3), "bytes": p2["bytes"] / its,
                           "gbs": round(p2["bytes"] / max(p2["ms"] * 1e-3, 1e-12) / 1e9, 1)},
                "tiles": ctx.plan_info().get("tiles", 0),
                "cg_iterations": its, "cg_iteration_us": round(1e3 * cg / its, 3), "lambda": rep["lambda_final"],
                "rank": rank}
        cal, cal_src = fetch_calibration()
        for pm in sorted(ROOT.glob("profiles/*_pmc_sp_product.json")):
            pj = json.loads(pm.read_text())
            if abs(pj.get("bytes_per_launch_algorithmic", -1) - out["bytes_per_launch"]) < 1e-6 * out["bytes_per_launch"]:
                f = pj.get("fetch_bytes_per_launch_raw")
                w = pj.get("write_bytes_per_launch")
                if cal is not None and f is not None and w is not None:
                    # the calibrated factors of 8-B-per-lane reads / writes (the kernels' dominant width)
                    f = f / cal["factor_fetch_read8"]
                    w = w / cal["factor_write8"]
                    out["traffic"] = f + w
                    out["traffic_calibration"] = cal_src
                else:
                    out["traffic"] = pj["traffic_bytes_per_launch"]
                out["traffic_source"] = pm.name
                if survey:
                    out["traffic_over_survey_bytes"] = round(out["traffic"] / survey, 3)
        return out
    if "pcg_product" in stats:
        pp = stats["pcg_product"]
        its = max(pp["launches"], 1)
        gbs = pp["bytes"] / max(pp["ms"] * 1e-3, 1e-12) / 1e9
        mf = "mf_lin" in stats
        cg = sum(stats[k]["ms"] for k in ("pcg_product", "pcg_heavy", "pcg_update") if k in stats)
        out = {"bound": "hbm", "kernel": "k_mf_product" if mf else "k_pcg_product", "achieved": round(gbs, 1),
               "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
               "traffic_unit": "bytes per launch", "bytes_per_launch": pp["bytes"] / its, "launches": its,
               "avg_active_launch_us": round(1e3 * pp["ms"] / its, 3),
               "cg_iterations": its, "cg_iteration_us": round(1e3 * cg / its, 3), "lambda": rep["lambda_final"],
               "rank": rank}
        for pm in sorted(ROOT.glob("profiles/*_pmc_*product.json")):
            pj = json.loads(pm.read_text())
            if abs(pj.get("bytes_per_launch_algorithmic", -1) - out["bytes_per_launch"]) < 1e-6 * out["bytes_per_launch"]:
                out["traffic"] = pj["traffic_bytes_per_launch"]
                out["traffic_source"] = pm.name
        return out
    return None


def factor_roofline(stats_f, rank):
    upd = stats_f["update"]
    achieved = upd["flops"] / (upd["ms"] * 1e-3) / 1e12
    traffic = None
    pmc = sorted(ROOT.glob("profiles/*_pmc_k_update.json"))
    if pmc:
        pj = json.loads(pmc[-1].read_text())
        if abs(pj.get("update_flops_per_factorization", -1) - upd["flops"]) < 1e-6 * upd["flops"]:
            traffic = pj["traffic_bytes_per_factorization"]
    return {"bound": "mfma", "kernel": "k_update", "achieved": round(achieved, 3),
            "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 4),
            "peak_sustained_measured": MFMA_F64_SUSTAINED_TFLOPS,
            "traffic": traffic, "traffic_unit": "bytes per factorization (all k_update launches)",
            "launches": upd["launches"], "avg_launch_us": round(1e3 * upd["ms"] / max(upd["launches"], 1), 3),
            "flops_per_factorization": upd["flops"], "rank": rank}


def timed_leg(prob, gpu, rank, world, backend, steps, warmup, label):
    """One more timed LM run in the bench line: the same plan choice and transport as the headline,
    `steps` LM iterations after `warmup`, max over ranks; CG iterations per trial and the product's
    roofline from a profiled trial."""
    ctx = capi.Context(gpu)
    try:
        if world > 1:
            from deftri import dist as ddist
            if backend == "nccl":
                ddist.init_rccl(ctx, rank, world)
            else:
                ctx.dist_set_transport(world, rank, ddist.torch_transport())
        t0 = time.perf_counter()
        ctx.upload(prob)
        info = ctx.plan_info()
        log(f"[rank {rank}] {label}: upload {time.perf_counter() - t0:.1f}s, {prob.summary()}")
        if warmup > 0:
            ctx.solve_lm(warmup)
        ctx.reset_state()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rep = ctx.solve_lm(steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
        t_max, _, _ = reduce_stats(dt, rep["iterations"], rep["trials_total"], world,
                                   "cuda" if backend == "nccl" else "cpu")
        stats = ctx.profile_trial(rep["lambda_final"])
        roof = product_roofline(stats, rep, ctx, rank)
        its = max(rep["iterations"], 1)
        out = {"value": its / t_max, "unit": "LM iterations/s", "ms_per_step": 1e3 * t_max / its, "steps": steps,
               "iterations": rep["iterations"], "unknowns": rep["n_unknowns"], "points": prob.n_points,
               "arap_edges": len(prob.arap_pair), "trials_per_iteration": round(rep["trials_total"] / its, 3),
               "cg_iterations_per_trial": round(rep["pcg_iterations"] / max(rep["pcg_trials"], 1), 2),
               "pcg_failed": rep["pcg_fallbacks"], "chi2_initial": rep["chi2_initial"], "chi2_final": rep["chi2_final"],
               "lambda_final": rep["lambda_final"], "plan": info["plan"], "cg_launches_per_iteration": info.get("cg_launches"),
               "parallelism": f"points{world}" if world > 1 else "single"}
        if roof:
            out.update({"cg_iteration_us": roof.get("cg_iteration_us"), "frac_survey": roof.get("frac_survey"),
                        "frac_design": roof.get("frac_design")})
        log(f"[rank {rank}] {label}: {out}")
        return out
    finally:
        ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=25, help="LM iterations timed (Simulation.yaml numberOfIterations: 25)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--trace-markers", action="store_true",
                    help="a tiny torch kernel right before and after the timed region (kernel-trace windows)")
    ap.add_argument("--corr", type=int, default=0, help="correspondences per keyframe (default: the workload's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--regime", choices=list(REGIMES), default="simulation",
                    help="c2: the weight regime (Simulation.yaml default; Drunkard / Realcolon weights and cameras)")
    ap.add_argument("--rounds", type=int, default=0, help="--workload deformation: cap the outer rounds (0: Simulation.yaml's)")
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5", "ba", "deformation"], default="c2",
                    help="c2: the headline (BASELINE.json metric); c3-c5: the multi-keyframe configs; ba: bundle adjustment")
    ap.add_argument("--pair-window", type=int, default=-1,
                    help="keyframe pairs: 0 every pair (the reference), w > 0 pairs at most w apart (default: the workload's)")
    ap.add_argument("--ba-points", type=int, default=500000)
    ap.add_argument("--ba-kfs", type=int, default=8)
    ap.add_argument("--ba-scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--lanes", type=int, default=0,
                    help="speculative LM lambda lanes (0: library default, 1: sequential trials)")
    ap.add_argument("--solver", choices=["pcg", "direct"], default="pcg",
                    help="LM step solver: block-Jacobi PCG (library default) or the multifrontal LDL^T")
    ap.add_argument("--plan", choices=["auto", "multifrontal", "iterative"], default="auto",
                    help="auto: multifrontal for one-GPU two-view PCG / any direct solve, iterative otherwise")
    ap.add_argument("--jacobian-fp32", action="store_true", help="iterative plan: fp32-stored ARAP Jacobians")
    ap.add_argument("--analytic", action="store_true",
                    help="closed-form ARAP/depth Jacobians (default: g2o numeric, the reference's arithmetic)")
    ap.add_argument("--sharded", action="store_true", help="kept for scripts: N > 1 is point-sharded by default")
    ap.add_argument("--strong", action="store_true", help="kept for scripts: N > 1 strong-scales by default")
    ap.add_argument("--weak", action="store_true",
                    help="N > 1: weak scaling instead (one problem of N x the correspondences; value in C2-equivalent "
                         "iterations/s) — the default is the BASELINE metric's fixed problem split over the N ranks")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the extra legs of the C2 line (the 500k x 2 north-star size, the Realcolon regime)")
    ap.add_argument("--c4-corr", type=int, default=WORKLOADS["c4"]["n"],
                    help="N > 1: correspondences per keyframe of the c4 leg (rehearsals on one GPU)")
    ap.add_argument("--replicas", action="store_true",
                    help="N > 1: N independent problems, one per GPU; value = per-problem LM it/s")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end arapOptimization timing")
    ap.add_argument("--cpu-full-iteration", action="store_true",
                    help="CPU baseline: time the oracle's whole first LM iteration (all trials)")
    args = ap.parse_args()
    global REGIME
    REGIME = args.regime

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    have_gpu = torch.cuda.is_available()
    if not have_gpu:
        raise SystemExit("bench.py needs a gfx950 GPU (no CPU path)")
    # one process per GPU (RCCL); DEFTRI_DIST_BACKEND=gloo + DEFTRI_GPU_OVERRIDE=0 rehearse several
    # ranks on one GPU (the sharded solve then moves its transfers through host memory over gloo)
    backend = os.environ.get("DEFTRI_DIST_BACKEND", "nccl")
    gpu = int(os.environ.get("DEFTRI_GPU_OVERRIDE", local))
    torch.cuda.set_device(gpu)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    red_dev = "cuda" if backend == "nccl" else "cpu"
    if args.workload == "ba":
        return main_ba(args, world, rank, gpu, backend)
    if args.workload == "deformation":
        return main_deformation(args, world, rank, gpu)

    wl = args.workload
    spec = WORKLOADS[wl]
    n = args.corr or spec["n"]
    window = args.pair_window if args.pair_window >= 0 else spec.get("window", 0)
    sharded = world > 1 and not args.replicas
    weak = sharded and args.weak
    n_build = n * world if weak else n        # weak: each rank's share is the workload's size
    plan = args.plan              # auto: the library's choice (iterative for PCG from 50k unknowns / sharded)
    t0 = time.perf_counter()
    prob, prob_map = build_workload(wl, n_build, 1 if sharded else 1 + rank, window)
    log(f"[rank {rank}] {wl} graph built in {time.perf_counter() - t0:.1f}s: {prob.summary()}")
    ctx = capi.Context(gpu)
    if sharded:
        from deftri import dist as ddist
        if backend == "nccl":
            ddist.init_rccl(ctx, rank, world)
        else:
            ctx.dist_set_transport(world, rank, ddist.torch_transport())
    ctx.set_plan(plan)
    ctx.set_jacobian_storage(1 if args.jacobian_fp32 else 0)
    ctx.set_linear_solver(args.solver)
    t0 = time.perf_counter()
    ctx.upload(prob)
    ctx.set_lm_lanes(args.lanes)
    info = ctx.plan_info()
    plan = info["plan"]
    log(f"[rank {rank}] upload ({info['plan']} plan) {time.perf_counter() - t0:.1f}s: {info}")
    analytic = args.analytic

    if args.warmup > 0:
        ctx.solve_lm(args.warmup, analytic=analytic)
    ctx.reset_state()

    if world > 1:
        dist.barrier()
    marker = torch.ones(1, device=f"cuda:{gpu}") if args.trace_markers else None
    if marker is not None:
        marker.mul_(2.0)                  # a kernel trace's window start (tools/trace_gaps.py --window mul)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rep = ctx.solve_lm(args.steps, analytic=analytic)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if marker is not None:
        marker.mul_(2.0)                  # ... and end (outside the timed region)
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    log(f"[rank {rank}] {rep['iterations']} iterations / {rep['trials_total']} trials in {dt * 1e3:.1f} ms; "
        f"chi2 {rep['chi2_initial']:.6e} -> {rep['chi2_final']:.6e}; lambda {rep['lambda_final']:.3e}; "
        f"pcg {rep['pcg_trials']} / failed {rep['pcg_fallbacks']}, {rep['pcg_iterations']} CG iterations")
    iters = rep["iterations"]
    if iters != args.steps:
        log(f"[rank {rank}] WARNING: LM terminated after {iters} of {args.steps} iterations")
    # one problem (sharded): every rank ran the same iterations, the job takes the slowest rank;
    # replicas: the slowest rank's time for its own problem (value = per-problem rate, never a sum)
    t_max, _, _ = reduce_stats(dt, iters, rep["trials_total"], world, red_dev)
    value, ms_per_step = job_rate(t_max, iters, world if weak else 1)

    # profiled trial (HIP events on the solver stream) at the final lambda of the timed run (a
    # collective on a sharded context: each rank times its own part of the same trial)
    stats = ctx.profile_trial(rep["lambda_final"])
    roofline = product_roofline(stats, rep, ctx, rank) if args.solver == "pcg" else None
    roofline_f, stats_f = None, None
    if plan == "multifrontal" and not sharded:
        if args.solver == "pcg":
            ctx.set_linear_solver("direct")
            stats_f = ctx.profile_trial(rep["lambda_final"])
            ctx.set_linear_solver(args.solver)
        else:
            stats_f = stats
        roofline_f = factor_roofline(stats_f, rank)
    if roofline is None:
        roofline = roofline_f
    trial_ms = {k: round(v["ms"], 4) for k, v in sorted(stats.items(), key=lambda kv: -kv[1]["ms"])}

    cpu = None
    trials_per_it = rep["trials_total"] / max(iters, 1)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        t0 = time.perf_counter()
        if wl == "c2":
            # the oracle eliminates in a nested-dissection order of the same problem (the host-only
            # analysis of the multifrontal plan): SimplicialLDLT's fill at C2 needs a good ordering
            if plan == "multifrontal":
                order = ctx.vertex_order()
            else:
                with capi.Context(-1) as hc:
                    hc.analyse(prob)
                    order = hc.vertex_order()
            cpu = cpu_baseline(prob, order, trials_per_it, args.cpu_full_iteration)
        else:
            cpu = cpu_baseline_sample(wl, window, {"c3": 400, "c4": 400, "c5": 300}[wl], trials_per_it)
        log(f"cpu baseline {time.perf_counter() - t0:.1f}s: {cpu}")

    e2e = None
    if world == 1 and not args.no_e2e and wl == "c2" and REGIME == "simulation" and n == 100000:
        def configure(c):
            c.set_plan(args.plan)
            c.set_jacobian_storage(1 if args.jacobian_fp32 else 0)
            c.set_linear_solver(args.solver)
            c.set_lm_lanes(args.lanes)
        e2e = end_to_end(gpu, prob_map, configure)
        log(f"end-to-end arapOptimization: {e2e}")

    legs_500k, regimes, legs_c4 = None, None, None
    headline = wl == "c2" and REGIME == "simulation" and n == 100000 and not args.replicas and not weak
    if headline and not args.no_legs and args.solver == "pcg":
        ctx.close()
        ctx = None
        p5 = build_problem(500000, 1)[0]
        legs_500k = timed_leg(p5, gpu, rank, world, backend, args.steps, min(args.warmup, 2), "500k x 2")
        legs_500k["correspondences_per_keyframe"] = 500000
        legs_500k["scaling"] = "strong" if world > 1 else "single"
        del p5
        if world > 1:
            # C4 (8 keyframes x 500k, all 28 pairs) point-sharded over the same ranks: the multi-pair
            # graph's sharded chain, a few LM iterations
            pc4, _ = build_workload("c4", args.c4_corr, 1, 0)
            legs_c4 = timed_leg(pc4, gpu, rank, world, backend, min(args.steps, 3), 1, "C4")
            legs_c4["workload"] = ("C4: " if args.c4_corr == WORKLOADS["c4"]["n"] else f"C4-slice-{args.c4_corr}x8: ") + \
                WORKLOADS["c4"]["desc"]
            legs_c4["scaling"] = "strong"
            del pc4
        if world == 1:
            pr, _ = build_problem(100000, 1, "realcolon")
            regimes = {"realcolon": timed_leg(pr, gpu, rank, world, backend, args.steps, min(args.warmup, 2),
                                              "C2 realcolon")}
            regimes["realcolon"]["weights"] = "Realcolon.yaml: rep 1, arap 0.1, DepthWeight 0.001 (sigma_d 1e-6 m), KB8 d0..d3"
            del pr

    if rank == 0:
        workload = (("C2" if n == 100000 else f"two-view-{n}") + ("" if REGIME == "simulation" else f"-{REGIME}")) if wl == "c2" else \
            (wl.upper() if n == spec["n"] else f"{wl.upper()}-slice-{n}x{spec['k']}")
        if weak:
            workload += f" x {world} (one problem of {n_build} correspondences per keyframe, point-sharded: {n} per GPU)"
        out = {
            "metric": (BASELINE_METRIC if REGIME == "simulation" else f"LM iterations/sec + ms/iter at 100k corr x 2 views, {REGIME} weights")
            if wl == "c2" else f"LM iterations/sec + ms/iter, {wl.upper()}: {spec['desc']}",
            "value": value, "unit": "LM iterations/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "weak" if (world > 1 and (weak or not sharded)) else "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": workload, "correspondences_per_keyframe": n, "keyframes": spec["k"],
                       "pairs": prob.n_pairs, "pair_window": window,
                       "points": prob.n_points, "arap_edges": len(prob.arap_pair), "unknowns": rep["n_unknowns"],
                       "plan": info["plan"], "jacobian_storage": "fp32" if info.get("jacobian_fp32") else "fp64",
                       "jacobians": "analytic" if analytic else "g2o numeric (reference)",
                       "step_solver": args.solver,
                       "trials_per_iteration": round(trials_per_it, 3),
                       "ms_per_trial": round(ms_per_step / max(trials_per_it, 1e-9), 3),
                       "pcg_trials": rep["pcg_trials"], "pcg_failed_or_fallback": rep["pcg_fallbacks"],
                       "cg_iterations_per_pcg_trial": round(rep["pcg_iterations"] / max(rep["pcg_trials"], 1), 2),
                       "pcg_continuations_per_trial": round(rep.get("pcg_continuations", 0) / max(rep["trials_total"], 1), 3),
                       "ms_per_cg_iteration_profiled": round(roofline["cg_iteration_us"] / 1e3, 4)
                       if roofline and "cg_iteration_us" in roofline else None,
                       "chi2_initial": rep["chi2_initial"], "chi2_final": rep["chi2_final"],
                       "lambda_final": rep["lambda_final"],
                       "own_rows_rank0": info.get("own_rows"), "halo_rows_rank0": info.get("halo_rows"),
                       "parallelism": (f"points{world}" if sharded else f"replicas{world}") if world > 1 else "single",
                       "value_semantics": "one problem, all ranks" if (world == 1 or (sharded and not weak))
                       else ("LM iterations/s of the N x sized problem x N (C2-equivalent iterations/s)" if weak
                             else "per-problem LM it/s of N independent problems (not summed)"),
                       "cg_launches_per_iteration": info.get("cg_launches"),
                       "cg_collectives_per_iteration": info.get("cg_collectives"),
                       "lm_control": "device" if os.environ.get("DEFTRI_DEVICE_LM") and not os.environ.get("DEFTRI_HOST_LM") and not sharded else "host"},
            "roofline": roofline,
            "roofline_factorization": roofline_f if roofline is not roofline_f else None,
            "cpu_baseline": cpu,
            "breakdown_ms": {"total": rep["ms_total"], "linearize": rep["ms_linearize"], "pcg": rep["ms_pcg"]},
            "trial_kernel_ms": trial_ms,
            "factorization_trial_kernel_ms": ({k: round(v["ms"], 3) for k, v in sorted(stats_f.items(), key=lambda kv: -kv[1]["ms"])}
                                              if stats_f is not None and stats_f is not stats else None),
            "end_to_end_arap_optimization": e2e,
            "north_star_500k": legs_500k,
            "c4": legs_c4,
            "regimes": regimes,
        }
        print(json.dumps(out), flush=True)
    if ctx is not None:
        ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
