"""The render kernel's exact fast divisions give IEEE division's bits.

The kernel replaces the 11-instruction correctly rounded f32 division with a refined hardware
reciprocal (v_rcp_f32 + one fma Newton step) and Markstein's correction wherever a correctly rounded
reciprocal is at hand.  The reciprocal is a property of this hardware, so it is pinned exhaustively on
the device: every f32 of its guarded range, both signs.  Division by the constants pi and tau is
checked for every f32 dividend, and the fast sqrt (v_sqrt_f32 + the ±1 ulp correction
without the range handling) for every f32.  Markstein's correction (a published theorem) is sampled on 2^32
pairs inside its guards, and the guarded helpers (their IEEE fallbacks included) on 2^30 pairs of any
kind: zeros, subnormals, extremes, infinities and NaN.  Counting happens on the device
(rtw_device_check_division); zero mismatches are required."""
import ctypes as C

import pytest

from raytracinginaweekend_amd import _native as N

pytestmark = pytest.mark.gpu


def _check(test, base, n, seed=0):
    bad, first = C.c_uint64(), C.c_uint64()
    N.check(N.lib().rtw_device_check_division(0, test, base, n, seed, C.byref(bad), C.byref(first)))
    return bad.value, first.value


def _f32_bits(sign, biased_exp):
    return (sign << 31) | (biased_exp << 23)


@pytest.mark.parametrize("sign", [0, 1])
def test_refined_reciprocal_every_f32_in_range(sign):
    # RTW_RCP_LO = 2^-100 .. RTW_RCP_HI = 2^100: biased exponents 27 .. 227 (2^100 itself included)
    lo = _f32_bits(sign, 27)
    hi = _f32_bits(sign, 227) + 1
    bad, first = _check(0, lo, hi - lo)
    assert bad == 0, f"rcp_nr differs from 1/b on {bad} inputs, first bits {lo + first:#010x}"


def test_division_by_pi_and_tau_every_f32():
    bad, first = _check(1, 0, 1 << 32)
    assert bad == 0, f"div_c differs on {bad} inputs, first bits {first:#010x}"


def test_markstein_inside_guards():
    bad, first = _check(2, 0, 1 << 32, seed=0x5EED)
    assert bad == 0, f"{bad} mismatches, first case {first}"


def test_guarded_helpers_any_input():
    bad, first = _check(3, 0, 1 << 30, seed=0xD1CE)
    assert bad == 0, f"{bad} mismatches, first case {first}"


def test_sqrt_every_f32():
    # sqrt_x on every bit pattern, sqrt_nr (no range handling) on [2^-96, FLT_MAX]
    bad, first = _check(4, 0, 1 << 32)
    assert bad == 0, f"sqrt_x / sqrt_nr differ from sqrtf on {bad} inputs, first bits {first:#010x}"


def test_triangle_t_without_guard():
    """tri_t_mk (the triangle test's t = num / denom by rcp_nr + Markstein, no guard): for
    divisors in tri_test's range (1e-4 < |denom| <= ~1) and dividends of any kind, equal to IEEE
    division whenever the quotient reaches ts = 0.001, and below ts whenever IEEE's is."""
    bad, first = _check(5, 0, 1 << 31, seed=0x7E57)
    assert bad == 0, f"{bad} mismatches, first case {first}"


def test_texel_channel_every_byte():
    """tex255 (an image texel's channel, texture.rs:30-31 `as f32 / 255.0`) by Markstein's correction
    without a guard: equal to the IEEE division for all 256 byte values."""
    bad, first = _check(6, 0, 256)
    assert bad == 0, f"{bad} mismatches, first byte {first}"
