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


def test_checker_sign():
    """CheckerTexture's `sines < 0` (texture.rs:33-40): the kernel decides it from rtw_sinf's
    quadrant reduction when that is unambiguous, else from the sines; the oracle multiplies the
    f32 sines (RN at each product)."""
    rng = np.random.default_rng(77)
    n = 600_000
    parts = [
        rng.uniform(-2000, 2000, (n, 3)).astype(np.float32),                  # pos * 10 on the ground sphere
        rng.uniform(-4, 4, (n, 3)).astype(np.float32),
        _random_floats(rng, 3 * n).reshape(n, 3),
    ]
    # floats next to multiples of pi/2 (small remainders), tiny / zero / subnormal / huge / non-finite
    k = np.arange(-400_000, 400_000, 7, dtype=np.float64)
    near = (k * (np.pi / 2)).astype(np.float32)
    near = np.concatenate([near, np.nextafter(near, np.float32(np.inf)), np.nextafter(near, np.float32(-np.inf))])
    m = len(near)
    parts.append(np.stack([near, rng.permutation(near), rng.uniform(-3, 3, m).astype(np.float32)], 1))
    sp = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-38, -3e-39, 2.0**-31, -(2.0**-30), 2.0**-29, 1e-20, -1e-30,
                   2.0**19, -(2.0**19), 2.0**19 - 0.03125, 3.4e38, np.inf, -np.inf, np.nan, 1.0, -1.0, 3.1415927,
                   -3.1415927, 1.5707964], np.float32)
    g = np.stack(np.meshgrid(sp, sp, sp, indexing="ij"), -1).reshape(-1, 3)
    parts.append(g)
    xyz = np.ascontiguousarray(np.concatenate(parts).astype(np.float32))
    out = np.empty(len(xyz), np.int32)
    N.check(N.lib().rtw_device_eval_checker(0, xyz.ctypes.data_as(C.POINTER(C.c_float)), len(xyz),
                                            out.ctypes.data_as(C.POINTER(C.c_int32))))
    s = O.eval_scalar(3, xyz.reshape(-1)).reshape(-1, 3)
    with np.errstate(all="ignore"):
        want = ((s[:, 0] * s[:, 1]) * s[:, 2] < np.float32(0)).astype(np.int32)
    bad = np.nonzero(out != want)[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, first {xyz[bad[:5]]}"


def test_uv_functions_dense():
    """The render kernel's acosf / atan2f (div_x / sqrt_x inside, rtw_device.hip d_acosf / d_atan2f)
    against the host restatements: every f32 bit pattern in [-1, 1] of a 4M-value stride sample for
    acos (all of its branches and their edges), and atan2 pairs whose ratios sit on both sides of
    atanf's branch points (7/16, 11/16, 19/16, 39/16, 2^+-25) and of the 2^+-60 shortcuts."""
    rng = np.random.default_rng(123)
    bits = np.arange(0, 0x3F800001, 253, dtype=np.uint64).astype(np.uint32)
    a = bits.view(np.float32)
    a = np.concatenate([a, -a, np.float32([0.5, -0.5, 2.0**-26, -(2.0**-26), 2.0**-25])])
    assert_bit_identical(_device(0, a), O.eval_scalar(0, a), "acos dense")
    r = np.float32([7 / 16, 11 / 16, 19 / 16, 39 / 16, 2.0**25, 2.0**-29, 2.0**60, 2.0**-60, 1.0])
    x = np.exp2(rng.uniform(-40, 40, 60_000)).astype(np.float32) * rng.choice([-1, 1], 60_000).astype(np.float32)
    ys = []
    xs = []
    for q in r:
        for d in (-2, -1, 0, 1, 2):
            ratio = np.float32(q) * np.float32(1 + d * 2.0**-23)
            ys.append((x * ratio).astype(np.float32) * rng.choice([-1, 1], len(x)).astype(np.float32))
            xs.append(x)
    y = np.concatenate(ys)
    xx = np.concatenate(xs)
    assert_bit_identical(_device(1, y, xx), O.eval_scalar(1, y, xx), "atan2 branch points")
