"""The f32 elementary functions of the shared spec (include/rtw_scalar.h) against numpy f64
references rounded to f32: correctly rounded except double-rounding hard cases, and never more
than 1 ulp from the true value (the reference uses glibc, itself within 1 ulp)."""
import numpy as np
import pytest

from oracle import pyoracle as O


def ulp_diff(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -2**31 - a, a)
    b = np.where(b < 0, -2**31 - b, b)
    return np.abs(a - b)


def _check(got, want, name, exact_frac=0.9999):
    got = np.asarray(got, np.float32)
    want = np.asarray(want, np.float32)
    nan = np.isnan(want)
    assert np.array_equal(np.isnan(got), nan), f"{name}: NaN mismatch"
    d = ulp_diff(got[~nan], want[~nan])
    assert d.max() <= 1, f"{name}: max ulp {d.max()}"
    assert (d == 0).mean() >= exact_frac, f"{name}: only {(d == 0).mean():.6f} correctly rounded"


def test_acos():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-1, 1, 300000), [-1, 1, 0, -0.0, 0.5, -0.5, 1.0000001, -1.0000001]]).astype(np.float32)
    with np.errstate(invalid="ignore"):
        _check(O.eval_scalar(0, x), np.arccos(x.astype(np.float64)).astype(np.float32), "acos")


def test_atan2_values_and_special_cases():
    rng = np.random.default_rng(1)
    y = rng.uniform(-2, 2, 300000).astype(np.float32)
    x = rng.uniform(-2, 2, 300000).astype(np.float32)
    _check(O.eval_scalar(1, y, x), np.arctan2(y.astype(np.float64), x.astype(np.float64)).astype(np.float32), "atan2")
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf], np.float32)
    yy, xx = np.repeat(sp, len(sp)), np.tile(sp, len(sp))
    got = O.eval_scalar(1, yy, xx)
    want = np.arctan2(yy.astype(np.float64), xx.astype(np.float64)).astype(np.float32)  # C99 special cases
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_ln():
    rng = np.random.default_rng(2)
    x = np.concatenate([rng.uniform(0, 1, 300000), rng.uniform(0, 1e-30, 1000), [0.0, 1.0, np.inf, -1.0, 1e-45, 3e38]])
    x = x.astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        _check(O.eval_scalar(2, x), np.log(x.astype(np.float64)).astype(np.float32), "ln")


def test_sin():
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.uniform(-10, 10, 200000), rng.uniform(-3000, 3000, 100000), [0.0, -0.0, np.pi, 1e-30]])
    x = x.astype(np.float32)
    _check(O.eval_scalar(3, x), np.sin(x.astype(np.float64)).astype(np.float32), "sin")
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
