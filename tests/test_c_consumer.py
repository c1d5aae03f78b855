"""The C-ABI from a compiled C program (tests/c_consumer/consumer.c, gcc against include/deftri.h,
linked with libdeftri.so): the header is plain C, the entry points link, and a C caller gets the
same numbers as the Python binding.  CPU part: simulation, graph build, symbolic analysis; the GPU
part runs the map-level arapOptimization from C."""
import pathlib
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT

SRC = ROOT / "tests" / "c_consumer" / "consumer.c"


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = tmp_path_factory.mktemp("cc") / "consumer"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-O2", "-I", str(ROOT / "include"), str(SRC), "-o", str(out),
                    "-L", str(PKG), "-ldeftri", f"-Wl,-rpath,{PKG}", "-lm"], check=True)
    return out


def _run(exe, *args):
    r = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return {line.split()[0]: line.split()[1:] for line in r.stdout.splitlines()}


def test_c_consumer_host(exe):
    out = _run(exe)
    assert out["abi"] == ["8"] and "ok" in out
    P, Q, S, R, D, E = map(int, out["graph"])
    assert (P, Q, S, R, D) == (800, 1, 2, 800, 800) and E > 2000
    n_unk, nnz, mflop, nf, nl = out["plan"]
    assert int(n_unk) == 6 * Q + S + 3 * P
    assert int(nnz) > 0 and float(mflop) > 0 and int(nf) > 1 and int(nl) > 1


def test_c_consumer_matches_python_binding(exe):
    """The same simulation call through ctypes returns the values the C program printed."""
    from deftri import capi, sim
    out = _run(exe)
    i = np.arange(400)
    gx, gy = (i % 20) - 9.5, (i // 20) - 9.5
    f = np.float32
    orig = np.stack([f(0.004) * gx.astype(f) + f(0.0003) * np.sin(f(1.7) * i.astype(f)),
                     f(0.004) * gy.astype(f) + f(0.0003) * np.cos(f(2.3) * i.astype(f)),
                     f(0.2) + f(0.002) * np.sin(f(0.3) * gx.astype(f)) * np.cos(f(0.2) * gy.astype(f))], 1).astype(f)
    moved = orig.copy()
    moved[:, 0] += f(0.0005) * np.sin(f(0.9) * i.astype(f))
    moved[:, 1] += f(0.0025)
    moved[:, 2] += f(0.0005) * np.cos(f(1.1) * i.astype(f))
    uv1, uv2, d1, d2, q1, q2 = capi.sim_two_view(orig, moved, (-0.1, 0.02, 0.12), (0.14, 0.01, 0.06), sim.SIM_KB8,
                                                 sim.SIM_KB8, 1.0, 1, 3.0, (0.4, 1.7))
    # libm sinf/cosf vs numpy's float32 sin/cos may differ in the last ulp: compare to the 0.1 px grid
    assert abs(uv1[0, 0] - float(out["uv1_0"][0])) < 0.11 and abs(uv1[0, 1] - float(out["uv1_0"][1])) < 0.11
    assert abs(d2[0] - float(out["d2_0"][0])) < 1e-6


@pytest.mark.gpu
def test_c_consumer_gpu(exe):
    out = _run(exe, "gpu")
    it, trials, chi0, chi1 = int(out["lm"][0]), int(out["lm"][1]), float(out["lm"][2]), float(out["lm"][3])
    assert it >= 1 and trials >= it and chi1 < chi0
    assert float(out["update"][0]) > 0
    assert all(np.isfinite(float(v)) for v in out["tg"])
