"""Diagnostic: merged vs three-launch CG chain vs the oracle on the golden cases (prints trajectories)."""
import os, sys, json, pathlib
import multiprocessing as mp
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))


def run(env, q):
    os.environ.update(env)
    from deftri import capi
    from deftri.problem import Problem
    out = {}
    for g in sorted((ROOT / "tests/golden").iterdir()):
        if not (g / "problem.npz").exists():
            continue
        p = Problem.load(g / "problem.npz")
        with capi.Context(0) as c:
            c.set_plan("iterative")
            c.set_linear_solver("pcg", max_iterations=4096)
            c.upload(p)
            r = c.solve_lm(10, analytic=True)
            out[g.name] = dict(trials=r["trials_iter"][:10], chi=[float(x) for x in r["chi2_iter"][:10]],
                               pcg=r["pcg_iterations"], fb=r.get("pcg_fallbacks"), ptr=r.get("pcg_trials"), tt=r["trials_total"], launches=c.plan_info()["cg_launches"])
    q.put(out)


if __name__ == "__main__":
    cm = mp.get_context("spawn")
    res = {}
    for name, env in (("merged", {}), ("three", {"DEFTRI_SP_NO_MERGE": "1"})):
        q = cm.Queue()
        pr = cm.Process(target=run, args=(env, q)); pr.start()
        res[name] = q.get(timeout=300); pr.join()
    from oracle import oracle
    from deftri.problem import Problem
    for g in res["merged"]:
        p = Problem.load(ROOT / "tests/golden" / g / "problem.npz")
        ref = oracle.solve_lm(p, 10, analytic=True)["report"]
        res.setdefault("oracle", {})[g] = dict(trials=list(ref["trials_iter"][:10]), chi=[float(x) for x in ref["chi2_iter"][:10]])
    for g in res["merged"]:
        print(g)
        for k in ("merged", "three", "oracle"):
            print(" ", k, json.dumps(res[k][g]))
