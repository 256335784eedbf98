"""The device slab test divides with a per-ray reciprocal (Markstein); under the kernel's guards
it must return exactly IEEE a/b.  tests/native/markstein_check.c covers every divisor
significand with random dividends across the guarded exponent ranges."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_markstein_division_is_exact_under_guards(tmp_path):
    exe = tmp_path / "mk"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-mfma", "-o", str(exe),
                    os.path.join(HERE, "native", "markstein_check.c"), "-lm"], check=True)
    out = subprocess.run([str(exe), "16"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:]
    assert "mismatches=0" in out.stdout
