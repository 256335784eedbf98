/* Exhaustive-over-divisor check of the division used by the device slab tests
 * (rtw_device.hip mk_div / node_pass):
 *   y = RN(1/b); q = RN(a*y); r = fma(-b, q, a); q' = fma(r, y, q)
 * must equal RN(a/b) under the kernel's guards: range 1 (slab and rect tests, per-ray
 * reciprocals) 2^-60 <= |b| <= 2, 2^-84 <= |a| <= 2^40 (a = 0 gives a zero quotient whose sign may
 * differ; no comparison of the slab test sees it); range 2 (the shading and triangle divisions,
 * DESIGN §5.8) 2^-22 <= |b| <= 2^22, 2^-80 <= |a| <= 2^80.
 * (Markstein 1990; Handbook of Floating-Point Arithmetic, Thm. "Markstein".)
 * For every divisor significand (2^23) and a spread of exponents, test many dividends. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static uint64_t s = 0x9E3779B97F4A7C15ull;
static inline uint64_t nxt(void) { s ^= s << 7; s ^= s >> 9; return s; }

int main(int argc, char** argv) {
    const int per = argc > 1 ? atoi(argv[1]) : 24;
    uint64_t tested = 0, guarded_out = 0, bad = 0;
    for (uint32_t m = 0; m < (1u << 23); ++m) {
        for (int k = 0; k < per; ++k) {
            const uint64_t r = nxt();
            const int r2 = (int)((r >> 60) & 1u);                     /* range 2 for every other case */
            const int be = r2 ? (int)(r % 45) - 22 : (int)(r % 62) - 60; /* divisor exponent */
            const uint32_t bs = (uint32_t)((r >> 8) & 1u) << 31;
            const float b = u2f(bs | ((uint32_t)(be + 127) << 23) | m);
            const int ae = r2 ? (int)((r >> 9) % 161) - 80 : (int)((r >> 9) % 124) - 84; /* dividend exponent */
            const uint32_t am = (uint32_t)(r >> 20) & 0x7FFFFFu;
            const uint32_t as = (uint32_t)((r >> 50) & 1u) << 31;
            const float a = u2f(as | ((uint32_t)(ae + 127) << 23) | am);
            const float y = 1.0f / b;
            const float q = a * y;
            const float rr = fmaf(-b, q, a);
            const float q2 = fmaf(rr, y, q);
            if (!r2 && fabsf(b) > 2.0f) { ++guarded_out; continue; }
            if (r2 && fabsf(b) > 0x1p22f) { ++guarded_out; continue; }
            const float t = a / b;
            ++tested;
            if (f2u(t) != f2u(q2)) {
                if (bad < 10) printf("MISMATCH a=%a b=%a true=%a got=%a\n", a, b, t, q2);
                ++bad;
            }
        }
    }
    /* zeros are outside the guard (q' = +0 for a = -0, b > 0): the device falls back to a/b */
    printf("tested=%llu guarded_out=%llu mismatches=%llu\n", (unsigned long long)tested,
           (unsigned long long)guarded_out, (unsigned long long)bad);
    return bad ? 1 : 0;
}
