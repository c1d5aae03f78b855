"""The ARAP energy divides by the pair area through its reciprocal (csrc/kernels.hip adiv: Markstein's
sequence, one division per edge).  The claim that it keeps the bits of x / area — the reference's
arithmetic (g2oTypes.h:310-339) — is checked here with the same sequence in C on the host's IEEE FMA
(tools/micro/div_markstein.c): random operands over a wide exponent range, divisors near the pair
areas and with all-ones mantissas, signed zeros and exact quotients.  The device kernels' own
agreement with the oracle is the job of the GPU parity tests."""
import pathlib
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent


def test_markstein_division_is_correctly_rounded(tmp_path):
    exe = tmp_path / "div_markstein"
    cc = subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(ROOT / "tools/micro/div_markstein.c"), "-lm"],
                        capture_output=True, text=True)
    if cc.returncode != 0:
        pytest.skip("no C compiler: " + cc.stderr[-200:])
    out = subprocess.run([str(exe), "300000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout[-1000:]
    assert out.stdout.strip().endswith("bad 0 of 3600000")
