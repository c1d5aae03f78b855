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

Multi-GPU (N > 1): N independent C2 problems, one per GPU (weak scaling, no data-path collective):
with PCG steps a C2 LM iteration is ~3 ms and a CG iteration ~0.13 ms of latency-bound work, less than
the latency of the halo exchange and two all-reduces a point-sharded CG iteration would need
(DESIGN.md §7).  --sharded runs ONE C2 problem point-sharded over the N ranks with the multifrontal
LDL^T (DistPlan, csrc/symbolic.cpp: a subtree of the nested-dissection tree per rank, separator
fronts on the leading ranks; per LM trial RCCL send/recv of one packed contribution block, one
forward vector and one boundary solution per rank, all-reduce of chi2 / rho denominator / pivot
flags) — strong scaling.  The barrier and the max-over-ranks time use torch.distributed.

Printed roofline: the dominant kernel of the configured step solver.  PCG (default): the product,
HBM-bound — k_mf_product (matrix-free, the default where the plan fits: per local edge its
linearized J, W, vertex dofs and record, the incidence slots, own (z, p_prev) and (p, q); csrc/pcg.hip
PcgMfHost::product_bytes) or k_pcg_product (assembled H: repacked slot records, heavy slots;
PcgHost::product_bytes) — bytes per launch x active launches / their summed device time, against
8 TB/s; `traffic` from the committed rocprofv3 PMC pass when it matches the plan.  The factorization's k_update roofline (algorithmic flops / device time, FP64 peak 78.6
TFLOP/s, AMD's MI355X specification) is reported beside it as roofline_factorization.  Both from
profiled trials right after the timed region, HIP events on the solver's own stream.

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


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_problem(n, seed):
    return sim.two_view_problem(n, seed, REP_W, ARAP_W, DEPTH_SIGMA, return_map=True)


def end_to_end(ctx, m, n_it=25):
    """The drop-in call a caller of the reference's arapOptimization makes (g2oBundleAdjustment.cc:608,
    Simulation.yaml weights rep 1 / global 50 / arap 2e5, nIt 25): host graph build + upload (+ the
    symbolic analysis, or its cached plan when the graph structure is unchanged) + device LM +
    write-back, wall time.  `cold` on a fresh context, `warm` on one that holds the same structure's
    plan (what every later call of deformationOptimization's loop / NLopt evaluations sees)."""
    import copy
    out = {"n_iterations": n_it}
    for key, c in (("cold", capi.Context(ctx.device)), ("warm", ctx)):
        mm = copy.deepcopy(m)
        t0 = time.perf_counter()
        _, rep = c.arap_optimization(mm, REP_W, 50.0, ARAP_W, 1.0, 1.0, DEPTH_SIGMA, n_it)
        out[key + "_s"] = round(time.perf_counter() - t0, 3)
        out[key + "_lm_s"] = round(rep["ms_total"] * 1e-3, 3)
        out[key + "_iterations"] = rep["iterations"]
        if c is not ctx:
            c.close()
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
            "value": iters / t_max, "unit": "LM iterations/s", "n_gpus": world, "steps": args.steps,
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--corr", type=int, default=100000, help="correspondences per GPU (C2: 100k)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=["c2", "ba"], default="c2",
                    help="c2: the headline ARAP LM (BASELINE.json); ba: point-sharded bundle adjustment")
    ap.add_argument("--ba-points", type=int, default=500000)
    ap.add_argument("--ba-kfs", type=int, default=8)
    ap.add_argument("--ba-scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--lanes", type=int, default=0,
                    help="speculative LM lambda lanes (0: library default, 1: sequential trials)")
    ap.add_argument("--solver", choices=["pcg", "direct"], default="pcg",
                    help="LM step solver: block-Jacobi PCG with LDL^T fallback (library default) or the LDL^T")
    ap.add_argument("--analytic", action="store_true",
                    help="closed-form ARAP/depth Jacobians (default: g2o numeric, the reference's arithmetic)")
    ap.add_argument("--sharded", action="store_true",
                    help="N > 1: one C2 problem point-sharded over the ranks (LDL^T, strong scaling) instead of "
                         "N independent problems (the default)")
    ap.add_argument("--replicas", action="store_true", help="N > 1: independent problems (the default; kept for scripts)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end arapOptimization timing")
    ap.add_argument("--cpu-full-iteration", action="store_true",
                    help="CPU baseline: time the oracle's whole first LM iteration (all trials)")
    args = ap.parse_args()

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

    sharded = world > 1 and args.sharded
    t0 = time.perf_counter()
    prob, prob_map = build_problem(args.corr, 1 if sharded else 1 + rank)
    log(f"[rank {rank}] graph built in {time.perf_counter() - t0:.1f}s: {prob.summary()}")
    ctx = capi.Context(gpu)
    if sharded:
        from deftri import dist as ddist
        if backend == "nccl":
            ddist.init_rccl(ctx, rank, world)
        else:
            ctx.dist_set_transport(world, rank, ddist.torch_transport())
    t0 = time.perf_counter()
    ctx.upload(prob)
    ctx.set_lm_lanes(args.lanes)
    ctx.set_linear_solver(args.solver)
    log(f"[rank {rank}] upload + symbolic analysis {time.perf_counter() - t0:.1f}s")
    analytic = args.analytic

    if args.warmup > 0:
        ctx.solve_lm(args.warmup, analytic=analytic)
    ctx.reset_state()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rep = ctx.solve_lm(args.steps, analytic=analytic)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    log(f"[rank {rank}] {rep['iterations']} iterations / {rep['trials_total']} trials in {dt * 1e3:.1f} ms; "
        f"chi2 {rep['chi2_initial']:.6e} -> {rep['chi2_final']:.6e}")
    iters = rep["iterations"]
    if iters != args.steps:
        log(f"[rank {rank}] WARNING: LM terminated after {iters} of {args.steps} iterations")

    if sharded:      # one problem: every rank ran the same iterations; the job takes the slowest rank
        t_max, _, _ = reduce_stats(dt, iters, rep["trials_total"], world, red_dev)
        it_sum, tr_sum = iters, rep["trials_total"]
    else:
        t_max, it_sum, tr_sum = reduce_stats(dt, iters, rep["trials_total"], world, red_dev)

    # profiled trial (HIP events on the solver stream), at the final lambda of the timed run
    # (a collective on a sharded context: each rank times its own part of the same trial)
    stats = ctx.profile_trial(rep["lambda_final"])
    pcg_prof = None
    if "pcg_product" in stats:
        # PCG steps: the dominant kernel is the product (HBM-bound row gathers); the factorization's
        # update kernel is profiled too (fallback path, and the direct solver's roofline)
        pp = stats["pcg_product"]
        its = max(pp["launches"] - 1, 1)           # the last launch only runs the convergence test
        gbs = pp["bytes"] / max(pp["ms"] * 1e-3, 1e-12) / 1e9
        mf = "mf_lin" in stats                     # matrix-free product (b + diagonal blocks only)
        pcg_prof = {"bound": "hbm", "kernel": "k_mf_product" if mf else "k_pcg_product", "achieved": round(gbs, 1),
                    "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                    "traffic_unit": "bytes per launch", "bytes_per_launch": pp["bytes"] / its,
                    "launches": pp["launches"], "avg_launch_us": round(1e3 * pp["ms"] / max(pp["launches"], 1), 3),
                    "avg_active_launch_us": round(1e3 * pp["ms"] / its, 3),
                    "cg_iterations": its, "lambda": rep["lambda_final"], "rank": rank}
        for pm in sorted(ROOT.glob("profiles/*_pmc_*product.json")) if not sharded else []:
            pj = json.loads(pm.read_text())
            if abs(pj.get("bytes_per_launch_algorithmic", -1) - pcg_prof["bytes_per_launch"]) < 1e-6 * pcg_prof["bytes_per_launch"]:
                pcg_prof["traffic"] = pj["traffic_bytes_per_launch"]
                pcg_prof["traffic_source"] = pm.name
        ctx.set_linear_solver("direct")
        stats_f = ctx.profile_trial(rep["lambda_final"])
        ctx.set_linear_solver(args.solver)
    else:
        stats_f = stats
    upd = stats_f["update"]
    factor_flops = rep["factor_flops_total"] if sharded else rep["factor_flops"]
    achieved = upd["flops"] / (upd["ms"] * 1e-3) / 1e12
    # HBM bytes of k_update per factorization from the committed rocprofv3 PMC pass (tools/gpu_pmc.sh +
    # tools/pmc_summary.py), attached only when it was collected on this same plan
    traffic = None
    pmc = sorted(ROOT.glob("profiles/*_pmc_k_update.json"))
    if pmc and not sharded:
        pj = json.loads(pmc[-1].read_text())
        if abs(pj.get("update_flops_per_factorization", -1) - upd["flops"]) < 1e-6 * upd["flops"]:
            traffic = pj["traffic_bytes_per_factorization"]
    roofline_f = {"bound": "mfma", "kernel": "k_update", "achieved": round(achieved, 3),
                "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 4),
                "peak_sustained_measured": MFMA_F64_SUSTAINED_TFLOPS,
                "traffic": traffic, "traffic_unit": "bytes per factorization (all k_update launches)",
                "launches": upd["launches"],
                "avg_launch_us": round(1e3 * upd["ms"] / max(upd["launches"], 1), 3),
                "flops_per_factorization": upd["flops"], "rank": rank}
    roofline = pcg_prof if pcg_prof else roofline_f
    trial_ms = {k: round(v["ms"], 3) for k, v in sorted(stats.items(), key=lambda kv: -kv[1]["ms"])}
    factor_trial_ms = {k: round(v["ms"], 3) for k, v in sorted(stats_f.items(), key=lambda kv: -kv[1]["ms"])}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        t0 = time.perf_counter()
        cpu = cpu_baseline(prob, ctx.vertex_order(), rep["trials_total"] / max(iters, 1), args.cpu_full_iteration)
        log(f"cpu baseline {time.perf_counter() - t0:.1f}s: {cpu}")

    e2e = None
    if world == 1 and not args.no_e2e:
        e2e = end_to_end(ctx, prob_map)
        log(f"end-to-end arapOptimization: {e2e}")

    if rank == 0:
        ms_per_step = 1e3 * t_max / max(iters, 1)
        trials_per_it = tr_sum / max(it_sum, 1)
        out = {
            "metric": BASELINE_METRIC,
            "value": it_sum / t_max, "unit": "LM iterations/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "strong" if sharded or world == 1 else "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": "C2" if args.corr == 100000 else f"two-view-{args.corr}",
                       "correspondences": args.corr, "views": 2,
                       "points": prob.n_points, "arap_edges": len(prob.arap_pair), "unknowns": rep["n_unknowns"],
                       "fronts": rep["n_fronts"], "nnz_factor": rep["nnz_factor"],
                       "factor_gflop": round(factor_flops / 1e9, 3),
                       "jacobians": "analytic" if analytic else "g2o numeric (reference)",
                       "trials_per_iteration": round(trials_per_it, 3),
                       "ms_per_trial": round(ms_per_step / max(trials_per_it, 1e-9), 3),
                       "lm_lanes": rep["lanes"],
                       "step_solver": args.solver if not sharded else "direct (point-sharded LDL^T)",
                       "pcg_product": ("matrix-free" if "mf_lin" in stats else "assembled") if pcg_prof else None,
                       "pcg_trials": rep["pcg_trials"], "pcg_fallbacks": rep["pcg_fallbacks"],
                       "cg_iterations_per_pcg_trial": round(rep["pcg_iterations"] / max(rep["pcg_trials"], 1), 2),
                       "trials_executed_per_iteration": round(rep["trials_executed"] / max(iters, 1), 3),
                       "parallelism": (f"points{world}" if sharded else f"replicas{world}") if world > 1 else "single"},
            "roofline": roofline,
            "roofline_factorization": roofline_f if pcg_prof else None,
            "cpu_baseline": cpu,
            "breakdown_ms": {"total": rep["ms_total"], "linearize": rep["ms_linearize"],
                             "factor": rep["ms_factor"], "solve": rep["ms_solve"], "update": rep["ms_update"],
                             "note": "factor/solve/update of sequential trials only with DEFTRI_TRIAL_EVENTS=1",
                             "pcg": rep["ms_pcg"]},
            "trial_kernel_ms": trial_ms,
            "factorization_trial_kernel_ms": factor_trial_ms if pcg_prof else None,
            "end_to_end_arap_optimization": e2e,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
