"""The work-item decode divides by launch invariants with multiply-high (rtw_device.hip fastdiv_make /
fdiv, Granlund & Montgomery 1994 Thm 4.2 at N = 32).  The same integer recipe, restated here,
must give floor(n / d) for every n < 2^32: checked on boundary dividends of many divisors."""
import numpy as np


def fastdiv_make(d):
    s = 0
    while s < 32 and (1 << s) < d:
        s += 1
    m = ((((1 << s) - d) << 32) // d + 1) & 0xFFFFFFFF
    return m, s


def fdiv(n, m, s):
    t = (n * m) >> 32
    return (t + n) >> s


def test_fastdiv_matches_floor_division():
    rng = np.random.default_rng(3)
    divisors = list(range(1, 2050)) + [64 * 63, 64 * 64, 259_200, 2_073_600, 8_294_400, 2**31 - 1, 2**31, 2**32 - 1]
    divisors += [int(x) for x in rng.integers(1, 2**32, 300)]
    for d in divisors:
        m, s = fastdiv_make(d)
        ns = [0, 1, d - 1, d, d + 1, 2**32 - 1, 2**32 - 2] + [k * d + r for k in (1, 2, 1000, (2**32 - 1) // d)
                                                               for r in (-1, 0, 1) if 0 <= k * d + r < 2**32]
        ns += [int(x) for x in rng.integers(0, 2**32, 50)]
        for n in ns:
            assert fdiv(n, m, s) == n // d, (n, d)
