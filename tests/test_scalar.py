"""The f32 elementary functions of the shared spec (include/rtw_scalar.h) are glibc 2.35's acosf,
atan2f, sinf and logf restated bit for bit (the libm the reference's f32::acos / atan2 / sin / ln
call: vec3.rs:242-243, texture.rs:32,50, hittable.rs:328).  Checked here through the oracle's
evaluator against the committed libm vectors (tests/golden/libm_f32.npz, which include the inputs
where glibc is not correctly rounded) and against the live libm; tests/test_libm.py runs the
exhaustive comparison."""
import ctypes
import os

import numpy as np
import pytest

from oracle import pyoracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = np.load(os.path.join(HERE, "golden", "libm_f32.npz"))
FN = {"acosf": 0, "atan2f": 1, "logf": 2, "sinf": 3}


def _same_bits(got, want, name):
    got = np.asarray(got, np.float32)
    want = np.asarray(want, np.float32)
    nan = np.isnan(want)
    assert np.array_equal(np.isnan(got), nan), f"{name}: NaN mismatch"
    bad = np.nonzero(got[~nan].view(np.uint32) != want[~nan].view(np.uint32))[0]
    assert len(bad) == 0, f"{name}: {len(bad)} of {len(got)} differ"


@pytest.mark.parametrize("name", ["acosf", "sinf", "logf"])
def test_unary_matches_glibc_fixture(name):
    x, y = FIX[f"{name}_x"], FIX[f"{name}_y"]
    _same_bits(O.eval_scalar(FN[name], x), y, name)


def test_atan2_matches_glibc_fixture():
    _same_bits(O.eval_scalar(1, FIX["atan2f_y"], FIX["atan2f_x"]), FIX["atan2f_r"], "atan2f")


def test_fixture_holds_inputs_where_glibc_is_not_correctly_rounded():
    """The vectors must be able to tell glibc from a correctly rounded restatement."""
    with np.errstate(all="ignore"):
        cr = {"acosf": np.arccos, "sinf": np.sin, "logf": np.log}
        for name, f in cr.items():
            x, y = FIX[f"{name}_x"], FIX[f"{name}_y"]
            rn = f(x.astype(np.float64)).astype(np.float32)
            ok = ~np.isnan(y)
            assert (rn[ok].view(np.uint32) != y[ok].view(np.uint32)).sum() >= 1000, name
        rn = np.arctan2(FIX["atan2f_y"].astype(np.float64), FIX["atan2f_x"].astype(np.float64)).astype(np.float32)
        assert (rn.view(np.uint32) != FIX["atan2f_r"].view(np.uint32)).sum() >= 1000


def _live_libm():
    try:
        m = ctypes.CDLL("libm.so.6")
    except OSError:
        pytest.skip("no libm.so.6")
    for n in ("acosf", "sinf", "logf"):
        getattr(m, n).restype = ctypes.c_float
        getattr(m, n).argtypes = [ctypes.c_float]
    m.atan2f.restype = ctypes.c_float
    m.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
    return m


def test_live_libm_fresh_draws():
    m = _live_libm()
    rng = np.random.default_rng(12345)
    bits = lambda n: rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    with np.errstate(all="ignore"):
        x = np.concatenate([rng.uniform(-1, 1, 20000), bits(5000)]).astype(np.float32)
        _same_bits(O.eval_scalar(0, x), [m.acosf(float(v)) for v in x], "acosf")
        x = np.concatenate([rng.uniform(-3000, 3000, 20000), bits(5000)]).astype(np.float32)
        _same_bits(O.eval_scalar(3, x), [m.sinf(float(v)) for v in x], "sinf")
        x = np.concatenate([rng.integers(0, 2**24, 20000) * 2.0**-24, bits(5000)]).astype(np.float32)
        _same_bits(O.eval_scalar(2, x), [m.logf(float(v)) for v in x], "logf")
        y = np.concatenate([rng.uniform(-1, 1, 20000), bits(5000)]).astype(np.float32)
        x = np.concatenate([rng.uniform(-1, 1, 20000), bits(5000)]).astype(np.float32)
        _same_bits(O.eval_scalar(1, y, x), [m.atan2f(float(a), float(b)) for a, b in zip(y, x)], "atan2f")


def test_sin_keeps_sign_of_zero():
    z = O.eval_scalar(3, np.array([-0.0], np.float32))
    assert z.view(np.uint32)[0] == 0x80000000


@pytest.mark.parametrize("fn", [4, 5])
def test_div_sqrt_are_ieee(fn):
    rng = np.random.default_rng(4)
    a = rng.uniform(-5, 5, 100000).astype(np.float32)
    b = rng.uniform(-5, 5, 100000).astype(np.float32)
    got = O.eval_scalar(fn, a, b)
    with np.errstate(invalid="ignore"):
        want = (a / b) if fn == 4 else np.sqrt(a)
    assert np.array_equal(np.isnan(got), np.isnan(want))
    m = ~np.isnan(want)
    assert np.array_equal(got[m].view(np.uint32), want[m].view(np.uint32))
