"""Multifrontal plan (csrc/symbolic.cpp): ordering, boundary sets, child->parent maps, arena
offsets and task lists, executed by the test-only host emulator (deftri_debug_plan_solve) against a
dense solve of the oracle's H.  The device kernels execute these same task lists (test_gpu_parity)."""
import numpy as np
import pytest

from conftest import GOLDEN
from deftri import capi, sim
from deftri.problem import Problem
from oracle import oracle


@pytest.fixture(scope="module")
def host():
    return capi.Context(-1)


def check(host, p, lam_rel=1e-5, fwd_tol=1e-8):
    host.analyse(p)
    st = host.plan_stats()
    assert st["n_unknowns"] == p.n_unknowns and st["n_fronts"] > 0
    b, H, _ = oracle.linearize(p, analytic=True, dense=True)
    lam = lam_rel * np.abs(np.diag(H)).max()
    x = host.debug_plan_solve(H, lam, b)
    A = H + lam * np.eye(len(b))
    xr = np.linalg.solve(A, b)
    # backward error of the multifrontal solve, and forward error vs the dense LAPACK solve
    assert np.linalg.norm(A @ x - b) / (np.linalg.norm(A, 2) * np.linalg.norm(x)) < 1e-13
    assert np.linalg.norm(x - xr) / np.linalg.norm(xr) < fwd_tol
    return st


def test_plan_golden(host, golden_cases):
    for name in golden_cases:
        check(host, Problem.load(GOLDEN / name / "problem.npz"))


@pytest.mark.parametrize("n", [40, 700])
def test_plan_two_view(host, n):
    m, _ = sim.simulate_two_view(n=n, seed=2)
    p = host.build_graph(m, 1.0, 2e5, np.float32(0.003))
    st = check(host, p)
    assert st["n_levels"] >= 2


def test_plan_multi_view(host):
    m, _ = sim.simulate_multi_view(n=150, k=3, seed=3)
    p = host.build_graph(m, 1.0, 2e5, np.float32(0.003))
    assert p.n_pairs == 3 and p.n_scales == 6
    check(host, p)


def test_plan_small_lambda(host, golden_cases):
    check(host, Problem.load(GOLDEN / golden_cases[0] / "problem.npz"), lam_rel=1e-9, fwd_tol=1e-5)


def test_plan_scaling_is_subquadratic(host):
    """Nested dissection on the mesh plane: factor entries grow ~ n log n, not n^2."""
    sizes, nnz = [], []
    for n in (2000, 8000):
        m, _ = sim.simulate_two_view(n=n, seed=1, scale_scene=True, compact=True)
        p = host.build_graph(m, 1.0, 2e5, np.float32(0.003))
        host.analyse(p)
        sizes.append(p.n_unknowns); nnz.append(host.plan_stats()["nnz_factor"])
    growth = np.log(nnz[1] / nnz[0]) / np.log(sizes[1] / sizes[0])
    assert growth < 1.5


def test_plan_lookahead_split(host, monkeypatch):
    """The optional LOOK/REST split of the outer updates (side-stream overlap, off by default)
    must factor exactly like the single trailing update."""
    monkeypatch.setenv("DEFTRI_LOOKAHEAD_MIN_M", "0")
    m, _ = sim.simulate_two_view(n=1500, seed=5, scale_scene=True, compact=True)   # root front s = 288 > one outer block
    p = host.build_graph(m, 1.0, 2e5, np.float32(0.003))
    check(host, p)
