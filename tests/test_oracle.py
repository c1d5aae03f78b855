"""Oracle (CPU restatement of the reference LM path) — formula-level pins and golden regression.

The reference cannot be built or run here (Eigen/g2o/Sophus/OpenCV/Open3D/Qhull absent),
and it ships no tests or golden vectors for this path, so the oracle is pinned by independent
cross-checks of each formula it restates: KB8 projection and its Jacobian (finite differences),
SE3Quat::exp (Rodrigues via scipy), g2o's numeric Jacobians vs the analytic ones, the sparse
LDL^T vs a dense solve, and the g2o LM acceptance rule.
"""
import json

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

from conftest import GOLDEN
from deftri import sim
from deftri.problem import Problem
from oracle import oracle
import ctypes as C


def _lib():
    return oracle.lib()


def kb8_proj(k, p):
    uv = np.zeros(2, np.float32)
    pf = np.asarray(p, np.float32)
    _lib().oracle_kb8_project(k.ctypes.data_as(C.POINTER(C.c_float)), pf.ctypes.data_as(C.POINTER(C.c_float)),
                              uv.ctypes.data_as(C.POINTER(C.c_float)))
    return uv


def kb8_jac(k, p):
    J = np.zeros(6, np.float32)
    pf = np.asarray(p, np.float32)
    _lib().oracle_kb8_project_jac(k.ctypes.data_as(C.POINTER(C.c_float)), pf.ctypes.data_as(C.POINTER(C.c_float)),
                                  J.ctypes.data_as(C.POINTER(C.c_float)))
    return J.reshape(2, 3)


@pytest.mark.parametrize("kb8", [sim.SIM_KB8, sim.REALCOLON_KB8])
def test_kb8_project_matches_formula(kb8):
    rng = np.random.default_rng(0)
    P = np.c_[rng.uniform(-0.3, 0.3, (50, 2)), rng.uniform(0.2, 1.0, 50)].astype(np.float32)
    ref = sim.kb8_project(kb8, P)
    got = np.array([kb8_proj(kb8, p) for p in P])
    assert np.abs(got - ref).max() < 1e-3          # fp32 libm differences only


@pytest.mark.parametrize("kb8", [sim.SIM_KB8, sim.REALCOLON_KB8])
def test_kb8_jacobian_finite_differences(kb8):
    rng = np.random.default_rng(1)
    k64 = kb8.astype(np.float64)

    def proj64(p):
        r = np.hypot(p[0], p[1]); th = np.arctan2(r, p[2]); psi = np.arctan2(p[1], p[0])
        rr = th + k64[4] * th ** 3 + k64[5] * th ** 5 + k64[6] * th ** 7 + k64[7] * th ** 9
        return np.array([k64[0] * rr * np.cos(psi) + k64[2], k64[1] * rr * np.sin(psi) + k64[3]])
    for _ in range(20):
        p = np.r_[rng.uniform(-0.3, 0.3, 2), rng.uniform(0.2, 1.0)]
        J = kb8_jac(kb8, p).astype(np.float64)
        h = 1e-6
        Jn = np.stack([(proj64(p + h * e) - proj64(p - h * e)) / (2 * h) for e in np.eye(3)], 1)
        assert np.abs(J - Jn).max() <= 1e-3 * np.abs(Jn).max()


def test_se3_exp_rodrigues():
    rng = np.random.default_rng(2)
    for scale in (1e-7, 1e-3, 0.5, 2.0):
        u = rng.normal(size=6) * scale
        out = np.zeros(7)
        _lib().oracle_se3_exp(u.ctypes.data_as(C.POINTER(C.c_double)), out.ctypes.data_as(C.POINTER(C.c_double)))
        q = out[:4]
        R = Rotation.from_quat(q).as_matrix()
        Rr = Rotation.from_rotvec(u[:3]).as_matrix()
        assert np.abs(R - Rr).max() < 1e-9 * max(1.0, scale) + 1e-12
        th = np.linalg.norm(u[:3]); W = np.array([[0, -u[2], u[1]], [u[2], 0, -u[0]], [-u[1], u[0], 0]])
        V = np.eye(3) + (1 - np.cos(th)) / th ** 2 * W + (th - np.sin(th)) / th ** 3 * W @ W if th > 1e-5 else \
            np.eye(3) + 0.5 * W + W @ W / 6
        assert np.abs(out[4:] - V @ u[3:]).max() < 1e-12 + 1e-9 * scale


def _golden(name):
    return Problem.load(GOLDEN / name / "problem.npz")


def test_numeric_vs_analytic_arap_jacobians(golden_cases):
    for name in golden_cases:
        p = _golden(name)
        Ja = oracle.arap_jacobians(p, analytic=True)
        Jn = oracle.arap_jacobians(p, analytic=False)
        scale = np.abs(Ja).max(axis=1, keepdims=True)
        assert np.abs(Ja - Jn).max() / scale.max() < 1e-5


def test_sparse_ldl_matches_dense(golden_cases):
    for name in golden_cases:
        p = _golden(name)
        b, H, _ = oracle.linearize(p, analytic=True, dense=True)
        lam = 1e-5 * np.abs(np.diag(H)).max()
        x = oracle.damped_solve(p, lam, b)
        xr = np.linalg.solve(H + lam * np.eye(len(b)), b)
        assert np.linalg.norm(x - xr) / np.linalg.norm(xr) < 1e-8


def test_hessian_is_jtj_symmetric_psd(golden_cases):
    p = _golden(golden_cases[0])
    b, H, _ = oracle.linearize(p, analytic=True, dense=True)
    assert np.abs(H - H.T).max() <= 1e-12 * np.abs(H).max()
    ev = np.linalg.eigvalsh(H / np.abs(H).max())
    assert ev.min() > -1e-10


def test_oracle_golden_regression(golden_cases):
    """The committed expected LM outputs (g2o numeric-Jacobian mode) are reproduced."""
    for name in golden_cases:
        p = _golden(name)
        exp = json.loads((GOLDEN / name / "expected.json").read_text())
        z = np.load(GOLDEN / name / "expected_lm.npz")
        r = oracle.solve_lm(p, exp["n_iterations"], analytic=False)
        R = r["report"]
        assert R["iterations"] == exp["iterations"] and R["trials_total"] == exp["trials_total"]
        np.testing.assert_allclose(R["chi2_iter"], z["chi2_iter"], rtol=1e-9)
        np.testing.assert_allclose(r["points"], z["points"], rtol=0, atol=1e-12)


def test_lm_rules(golden_cases):
    p = _golden(golden_cases[0])
    r = oracle.solve_lm(p, 8, analytic=True)
    chis = [r["report"]["chi2_initial"]] + r["report"]["chi2_iter"]
    assert all(b <= a for a, b in zip(chis, chis[1:]))      # accepted steps never increase chi2
    assert r["report"]["chi2_final"] == pytest.approx(chis[-1], rel=1e-12)
