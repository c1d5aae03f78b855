import os
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
PKG = ROOT / "triangulation-in-deformable-scenes_amd"
for p in (str(PKG), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; parity tests through the C-ABI")


def _ensure_built():
    import subprocess
    if not (PKG / "libdeftri.so").exists():
        subprocess.run(["make", "-s", "-C", str(PKG / "csrc"), "-j8"], check=True)
    if not (ROOT / "oracle" / "liboracle.so").exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def golden_cases():
    return sorted(p.name for p in GOLDEN.iterdir() if (p / "problem.npz").exists())


@pytest.fixture(scope="session")
def gpu_ctx():
    """One device context for the session, pinned to the multifrontal plan (the LDL^T / sliced
    matrix-free PCG suites); tests of the iterative plan set it explicitly and restore this."""
    from deftri import capi
    ctx = capi.Context(0)
    ctx.set_plan("multifrontal")
    yield ctx
    ctx.close()
