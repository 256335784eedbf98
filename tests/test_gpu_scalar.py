"""Device arithmetic vs host arithmetic for the shared scalar spec (include/rtw_scalar.h):
f32 division / sqrt must be correctly rounded on gfx950 and the f64-evaluated elementary
functions must give the same bits on both sides."""
import ctypes as C

import numpy as np
import pytest

from raytracinginaweekend_amd import _native as N
from oracle import pyoracle as O
from tests.parity import assert_bit_identical

pytestmark = pytest.mark.gpu


def _device(fn, a, b=None):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(a if b is None else b, np.float32)
    out = np.empty_like(a)
    f = C.POINTER(C.c_float)
    N.check(N.lib().rtw_device_eval_scalar(0, fn, a.ctypes.data_as(f), b.ctypes.data_as(f), len(a), out.ctypes.data_as(f)))
    return out


def _random_floats(rng, n):
    bits = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    x = bits.view(np.float32)
    return x


@pytest.mark.parametrize("fn,name", [(0, "acos"), (2, "ln"), (3, "sin"), (5, "sqrt")])
def test_unary(fn, name):
    rng = np.random.default_rng(fn)
    a = np.concatenate([
        rng.uniform(-1.2, 1.2, 400_000).astype(np.float32),
        rng.uniform(-3000, 3000, 200_000).astype(np.float32),
        _random_floats(rng, 400_000),
        np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 3.4e38], np.float32),
    ])
    assert_bit_identical(_device(fn, a), O.eval_scalar(fn, a), name)


@pytest.mark.parametrize("fn,name", [(1, "atan2"), (4, "div")])
def test_binary(fn, name):
    rng = np.random.default_rng(10 + fn)
    a = np.concatenate([rng.uniform(-2, 2, 500_000).astype(np.float32), _random_floats(rng, 500_000)])
    b = np.concatenate([rng.uniform(-2, 2, 500_000).astype(np.float32), _random_floats(rng, 500_000)])
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0], np.float32)
    a = np.concatenate([a, np.repeat(sp, len(sp))])
    b = np.concatenate([b, np.tile(sp, len(sp))])
    assert_bit_identical(_device(fn, a, b), O.eval_scalar(fn, a, b), name)
