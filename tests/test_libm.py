"""Exhaustive pin of the shared spec's elementary functions (include/rtw_scalar.h) against the
live platform libm, glibc 2.35 -- what the reference's f32::acos / atan2 / sin / ln call
(vec3.rs:242-243, texture.rs:32,50, hittable.rs:328):

  acosf, sinf, logf   every one of the 2^32 f32 bit patterns
  atan2f              2^28 pairs (random bits, [-2,2]^2, close magnitudes, unit normals) + specials
  sinsign             rtw_sin_sign_fast (the kernel's checker shortcut) against the sign of sinf,
                      every f32 where it decides

tests/native/libm_check.c does the work (about 90 s on 8 threads)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = tmp_path_factory.mktemp("libm") / "libm_check"
    subprocess.run(["gcc", "-O2", "-std=c11", "-march=x86-64-v3", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(HERE, "native", "libm_check.c"), "-lm", "-lpthread"], check=True)
    return str(exe)


def _threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return str(max(1, min(n, 16)))


@pytest.mark.parametrize("mode", ["acosf", "sinf", "logf", "sinsign"])
def test_every_f32(checker, mode):
    out = subprocess.run([checker, mode, _threads()], capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout[-2000:]
    assert "tested=4294967296 " in out.stdout and "mismatches=0" in out.stdout, out.stdout


def test_atan2f_pairs(checker):
    out = subprocess.run([checker, "atan2f", _threads(), str(1 << 28)], capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout[-2000:]
    assert "mismatches=0" in out.stdout, out.stdout
