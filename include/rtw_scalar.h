/*
 * rtw_scalar.h -- the scalar numeric specification shared by the HIP render kernel and the CPU
 * oracle.  Plain C99 (gcc) and HIP C++ (hipcc) from one text: every function is `RTW_HD`
 * (static inline, plus __host__ __device__ under hipcc).
 *
 * What lives here, and why it is shared rather than restated twice:
 *   1. xoroshiro128++ and the `rand 0.8.5` / `rand_distr 0.4.3` sampling semantics the reference
 *      hot path draws from (third-party crates, not vendored under /root/reference; see
 *      SURVEY.md §8(a) a22).  Restated from the published crate algorithms; pinned by the
 *      published rand_xoshiro test vector (tests/test_rng.py).
 *   2. The per-(pixel, sample) stream derivation ("ctr" mode) that makes the image independent
 *      of how pixels are spread over lanes, threads or GPUs.
 *   3. f32 elementary functions used on the device path (acos/atan2 for sphere uv
 *      `vec3.rs:241-249`, ln for volumes `hittable.rs:328`, sin for checker/marble
 *      `texture.rs:32,50`).  The reference calls the platform libm (glibc); these are evaluated in
 *      f64 and rounded once, i.e. correctly rounded except in double-rounding hard cases
 *      (probability ~2^-29 per call).  Tested against numpy f64 in tests/test_scalar.py.
 *   4. Rust-semantics helpers: f32::min/max (NaN-ignoring), saturating `as` casts, minmax.
 *
 * Everything else (geometry, BVH traversal, materials, the bounce loop) is implemented
 * separately by the oracle (oracle/rtw_oracle.c, a line-by-line C restatement) and by the
 * device kernel (raytracinginaweekend_amd/csrc/rtw_device.hip), so the parity tests compare
 * two independent implementations of the reference algorithm.
 *
 * Floating point contract: both sides compile with -ffp-contract=off and without fast-math;
 * f32 `/` and sqrtf are IEEE correctly rounded on both (hipcc default
 * -fhip-fp32-correctly-rounded-divide-sqrt).
 */
#ifndef RTW_SCALAR_H
#define RTW_SCALAR_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define RTW_HD static inline __host__ __device__
#else
#define RTW_HD static inline
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

#ifdef __cplusplus
extern "C++" {
#endif

/* ------------------------------------------------------------------------------------------ */
/* bit casts                                                                                   */
/* ------------------------------------------------------------------------------------------ */
RTW_HD uint32_t rtw_f2u(float f) { uint32_t u; __builtin_memcpy(&u, &f, 4); return u; }
RTW_HD float rtw_u2f(uint32_t u) { float f; __builtin_memcpy(&f, &u, 4); return f; }
RTW_HD uint64_t rtw_d2u(double f) { uint64_t u; __builtin_memcpy(&u, &f, 8); return u; }
RTW_HD double rtw_u2d(uint64_t u) { double f; __builtin_memcpy(&f, &u, 8); return f; }

RTW_HD int rtw_isnan(float x) { return x != x; }
RTW_HD int rtw_isnand(double x) { return x != x; }

/* ------------------------------------------------------------------------------------------ */
/* Rust f32 semantics                                                                          */
/* ------------------------------------------------------------------------------------------ */
/* f32::max / f32::min: IEEE maxNum/minNum (a NaN operand is ignored).  Equal operands
 * (including +0/-0) return `b`; the reference leaves that case to LLVM's lowering, this spec
 * fixes it so both sides agree bit for bit. */
RTW_HD float rtw_maxr(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    return (a > b) ? a : b;
}
RTW_HD float rtw_minr(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    return (a < b) ? a : b;
}
/* math.rs:18-27 clamp(low, high, value): NaN passes through. */
RTW_HD float rtw_clampr(float low, float high, float v) {
    return (v > high) ? high : ((v < low) ? low : v);
}
/* Rust `f as u32`: saturating, NaN -> 0. */
RTW_HD uint32_t rtw_f2u32_sat(float f) {
    if (!(f > 0.0f)) return 0u;                 /* NaN, <= 0 */
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}
/* Rust `f as i32`: saturating, NaN -> 0. */
RTW_HD int32_t rtw_f2i32_sat(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (-2147483647 - 1);
    return (int32_t)f;
}
/* Rust `f as u8`: saturating, NaN -> 0. */
RTW_HD uint8_t rtw_f2u8_sat(float f) {
    if (!(f > 0.0f)) return 0;
    if (f >= 255.0f) return 255;
    return (uint8_t)f;
}
/* Rust f32::signum: NaN -> NaN, +-0 -> +-1 (sign of zero kept), else +-1. */
RTW_HD float rtw_signum(float x) {
    if (x != x) return x;
    return (rtw_f2u(x) & 0x80000000u) ? -1.0f : 1.0f;
}

/* ------------------------------------------------------------------------------------------ */
/* xoroshiro128++  (rand_xoshiro 0.6.0 Xoroshiro128PlusPlus, the reference's TRng, common.rs:1) */
/* ------------------------------------------------------------------------------------------ */
typedef struct rtw_xoro {
    uint64_t s0, s1;
} rtw_xoro;

RTW_HD uint64_t rtw_rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

RTW_HD uint64_t rtw_xoro_next_u64(rtw_xoro* r) {
    const uint64_t s0 = r->s0;
    uint64_t s1 = r->s1;
    const uint64_t result = rtw_rotl64(s0 + s1, 17) + s0;
    s1 ^= s0;
    r->s0 = rtw_rotl64(s0, 49) ^ s1 ^ (s1 << 21);
    r->s1 = rtw_rotl64(s1, 28);
    return result;
}
/* next_u32 = low half of next_u64 (rand_xoshiro 0.6 `self.next_u64() as u32`). */
RTW_HD uint32_t rtw_xoro_next_u32(rtw_xoro* r) { return (uint32_t)rtw_xoro_next_u64(r); }

/* SeedableRng::from_seed([u8;16]): two little-endian u64 words; all-zero seed is replaced. */
RTW_HD rtw_xoro rtw_xoro_from_seed_bytes(const uint8_t seed[16]) {
    rtw_xoro r;
    uint64_t a = 0, b = 0;
    for (int i = 7; i >= 0; --i) a = (a << 8) | seed[i];
    for (int i = 15; i >= 8; --i) b = (b << 8) | seed[i];
    r.s0 = a;
    r.s1 = b;
    if ((a | b) == 0) { /* rand_xoshiro deal_with_zero_seed!: seed_from_u64(0) */
        uint64_t x = 0;
        for (int w = 0; w < 2; ++w) {
            uint64_t z = (x += 0x9E3779B97F4A7C15ull);
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z = z ^ (z >> 31);
            if (w == 0) r.s0 = z; else r.s1 = z;
        }
    }
    return r;
}

/* splitmix64: used to derive independent xoroshiro states (render streams). */
RTW_HD uint64_t rtw_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
RTW_HD uint64_t rtw_splitmix64_next(uint64_t* x) {
    *x += 0x9E3779B97F4A7C15ull;
    return rtw_mix64(*x);
}

/* "ctr" mode: one stream per (pixel, sample).  pixel = y*W + x of the full image, sample in
 * [0, spp).  The image is therefore independent of lane/thread/GPU assignment. */
RTW_HD uint64_t rtw_seed_key(uint64_t seed) { return rtw_mix64(seed ^ 0x5EED5EED5EED5EEDull); }
RTW_HD rtw_xoro rtw_sample_stream(uint64_t seed_key, uint32_t pixel, uint32_t sample) {
    uint64_t x = rtw_mix64((((uint64_t)pixel) << 32 | (uint64_t)sample) ^ seed_key);
    rtw_xoro r;
    r.s0 = rtw_splitmix64_next(&x);
    r.s1 = rtw_splitmix64_next(&x);
    if ((r.s0 | r.s1) == 0) r.s0 = 1;
    return r;
}
/* "ref" mode: one stream per worker thread, as rendering.rs:160,170 (StdRng -> from_rng),
 * deterministic here instead of from entropy. */
RTW_HD rtw_xoro rtw_thread_stream(uint64_t seed, uint32_t thread_id) {
    uint64_t x = rtw_mix64(seed ^ (0xA5A5A5A5ull << 32) ^ (uint64_t)thread_id);
    rtw_xoro r;
    r.s0 = rtw_splitmix64_next(&x);
    r.s1 = rtw_splitmix64_next(&x);
    if ((r.s0 | r.s1) == 0) r.s0 = 1;
    return r;
}

/* ------------------------------------------------------------------------------------------ */
/* rand 0.8.5 / rand_distr 0.4.3 distributions                                                  */
/* ------------------------------------------------------------------------------------------ */
/* Standard f32: (next_u32 >> 8) * 2^-24. */
RTW_HD float rtw_gen_f32(rtw_xoro* r) {
    const uint32_t v = rtw_xoro_next_u32(r) >> 8;
    return (1.0f / 16777216.0f) * (float)v;
}
/* UniformFloat value in [0,1): ((u32 >> 9) | exp(0)) - 1.0 */
RTW_HD float rtw_value0_1(uint32_t u) { return rtw_u2f((u >> 9) | 0x3F800000u) - 1.0f; }

typedef struct rtw_uniform {
    float low, scale;
} rtw_uniform;

/* Uniform::new(low, high) for f32 (UniformFloat::new): shrink scale until
 * scale*max_rand + low < high.  Caller guarantees low < high, both finite. */
RTW_HD rtw_uniform rtw_uniform_new(float low, float high) {
    const float max_rand = rtw_u2f((0xFFFFFFFFu >> 9) | 0x3F800000u) - 1.0f;
    float scale = high - low;
    for (;;) {
        const float top = scale * max_rand + low;
        if (!(top >= high)) break;
        scale = rtw_u2f(rtw_f2u(scale) - 1u);
    }
    rtw_uniform u;
    u.low = low;
    u.scale = scale;
    return u;
}
RTW_HD float rtw_uniform_sample(const rtw_uniform* u, rtw_xoro* r) {
    const float v = rtw_value0_1(rtw_xoro_next_u32(r));
    return v * u->scale + u->low;
}
/* Rng::gen_range(low..high) for f32 (UniformFloat::sample_single): redraw while res >= high. */
RTW_HD float rtw_gen_range_f32(float low, float high, rtw_xoro* r) {
    const float scale = high - low;
    for (;;) {
        const float v = rtw_value0_1(rtw_xoro_next_u32(r));
        const float res = v * scale + low;
        if (res < high) return res;
    }
}
/* Rng::gen_bool(p) via Bernoulli: p_int = (p * 2^64) as u64 (p < 1), draw u64 < p_int.
 * Only p = 0.5 occurs on the path (rendering.rs:79-80): p_int = 2^63. */
RTW_HD int rtw_gen_bool_half(rtw_xoro* r) { return rtw_xoro_next_u64(r) < 0x8000000000000000ull; }

/* Uniform::new(-1, 1) used by UnitDisc / UnitSphere / UnitBall: scale 2 needs no shrink
 * (2*(1-2^-23) - 1 < 1), so sample = v*2 + (-1). */
RTW_HD float rtw_uniform_m1_1(rtw_xoro* r) {
    const float v = rtw_value0_1(rtw_xoro_next_u32(r));
    return v * 2.0f + (-1.0f);
}
/* rand_distr::UnitDisc: rejection from the square, accept x1^2+x2^2 <= 1. */
RTW_HD void rtw_unit_disc(rtw_xoro* r, float out[2]) {
    float x1, x2;
    for (;;) {
        x1 = rtw_uniform_m1_1(r);
        x2 = rtw_uniform_m1_1(r);
        if (x1 * x1 + x2 * x2 <= 1.0f) break;
    }
    out[0] = x1;
    out[1] = x2;
}
/* rand_distr::UnitSphere (Marsaglia 1972). */
RTW_HD void rtw_unit_sphere(rtw_xoro* r, float out[3]) {
    for (;;) {
        const float x1 = rtw_uniform_m1_1(r);
        const float x2 = rtw_uniform_m1_1(r);
        const float sum = x1 * x1 + x2 * x2;
        if (sum >= 1.0f) continue;
        const float factor = 2.0f * __builtin_sqrtf(1.0f - sum);
        out[0] = x1 * factor;
        out[1] = x2 * factor;
        out[2] = 1.0f - 2.0f * sum;
        return;
    }
}
/* rand_distr::UnitBall: rejection from the cube, accept |x|^2 <= 1. */
RTW_HD void rtw_unit_ball(rtw_xoro* r, float out[3]) {
    float x1, x2, x3;
    for (;;) {
        x1 = rtw_uniform_m1_1(r);
        x2 = rtw_uniform_m1_1(r);
        x3 = rtw_uniform_m1_1(r);
        if (x1 * x1 + x2 * x2 + x3 * x3 <= 1.0f) break;
    }
    out[0] = x1;
    out[1] = x2;
    out[2] = x3;
}
/* gen_range(0..n) for u32 (UniformInt::sample_single_inclusive, Lemire widening multiply with
 * the "conservative" zone).  Used by SliceRandom::shuffle (perlin.rs:93-97). */
RTW_HD uint32_t rtw_gen_range_u32(uint32_t n, rtw_xoro* r) {
    const uint32_t range = n; /* high-1 - low + 1 */
    if (range == 0) return rtw_xoro_next_u32(r);
    const uint32_t lz = (uint32_t)__builtin_clz(range);
    const uint32_t zone = (range << lz) - 1u;
    for (;;) {
        const uint32_t v = rtw_xoro_next_u32(r);
        const uint64_t m = (uint64_t)v * (uint64_t)range;
        const uint32_t hi = (uint32_t)(m >> 32), lo = (uint32_t)m;
        if (lo <= zone) return hi;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* f32 elementary functions, evaluated in f64 and rounded once                                */
/* ------------------------------------------------------------------------------------------ */
#define RTW_PI_D 3.141592653589793115997963468544185161590576171875
#define RTW_PIO2_D 1.5707963267948965579989817342720925807952880859375
#define RTW_PIO6_D 0.52359877559829881565889309058547951281070709228515625
#define RTW_SQRT3_D 1.732050807568877193176604123436845839023590087890625
#define RTW_LN2_D 0.69314718055994528622676398299518041312694549560546875

/* atan on doubles; |error| ~ 1e-16 relative.  Reduction: |x|>1 -> pi/2 - atan(1/x);
 * x > tan(pi/12) -> pi/6 + atan((x*sqrt3 - 1)/(x + sqrt3)); then the Taylor series. */
RTW_HD double rtw_atan_d(double x) {
    const int neg = x < 0.0;
    if (neg) x = -x;
    int inv = 0;
    if (x > 1.0) {
        x = 1.0 / x;
        inv = 1;
    }
    double off = 0.0;
    if (x > 0.26794919243112270) {
        x = (x * RTW_SQRT3_D - 1.0) / (x + RTW_SQRT3_D);
        off = RTW_PIO6_D;
    }
    const double x2 = x * x;
    /* sum_{k=0..16} (-1)^k x^(2k+1) / (2k+1); |x| <= 0.268 -> truncation < 1e-20 */
    double p = -1.0 / 33.0;
    p = p * x2 + 1.0 / 31.0;
    p = p * x2 - 1.0 / 29.0;
    p = p * x2 + 1.0 / 27.0;
    p = p * x2 - 1.0 / 25.0;
    p = p * x2 + 1.0 / 23.0;
    p = p * x2 - 1.0 / 21.0;
    p = p * x2 + 1.0 / 19.0;
    p = p * x2 - 1.0 / 17.0;
    p = p * x2 + 1.0 / 15.0;
    p = p * x2 - 1.0 / 13.0;
    p = p * x2 + 1.0 / 11.0;
    p = p * x2 - 1.0 / 9.0;
    p = p * x2 + 1.0 / 7.0;
    p = p * x2 - 1.0 / 5.0;
    p = p * x2 + 1.0 / 3.0;
    double r = off + (x - x * x2 * p);
    if (inv) r = RTW_PIO2_D - r;
    return neg ? -r : r;
}

/* atan2f with C99 special cases (what Rust's f32::atan2 gets from libm). */
RTW_HD float rtw_atan2f(float y, float x) {
    if (x != x || y != y) return x + y;
    const int ysign = (rtw_f2u(y) >> 31) != 0;
    const int xsign = (rtw_f2u(x) >> 31) != 0;
    const float INF = rtw_u2f(0x7F800000u);
    if (y == 0.0f) {
        if (!xsign) return y;                      /* atan2(+-0, +x or +0) = +-0 */
        return ysign ? (float)-RTW_PI_D : (float)RTW_PI_D;
    }
    if (x == 0.0f) return ysign ? (float)-RTW_PIO2_D : (float)RTW_PIO2_D;
    if (x == INF || x == -INF) {
        if (y == INF || y == -INF) {
            const double a = xsign ? 3.0 * RTW_PI_D / 4.0 : RTW_PI_D / 4.0;
            return (float)(ysign ? -a : a);
        }
        if (!xsign) return ysign ? -0.0f : 0.0f;
        return ysign ? (float)-RTW_PI_D : (float)RTW_PI_D;
    }
    if (y == INF || y == -INF) return ysign ? (float)-RTW_PIO2_D : (float)RTW_PIO2_D;
    const double yd = y < 0.0f ? -(double)y : (double)y;
    const double xd = x < 0.0f ? -(double)x : (double)x;
    double a = rtw_atan_d(yd / xd);
    if (xsign) a = RTW_PI_D - a;
    return (float)(ysign ? -a : a);
}

/* acosf: 2*atan(sqrt((1-x)/(1+x))); |x| > 1 or NaN -> NaN. */
RTW_HD float rtw_acosf(float x) {
    if (x != x) return x;
    if (x > 1.0f || x < -1.0f) return rtw_u2f(0x7FC00000u);
    const double xd = (double)x;
    const double q = (1.0 - xd) / (1.0 + xd); /* x = -1 -> +inf -> atan = pi/2 */
    return (float)(2.0 * rtw_atan_d(__builtin_sqrt(q)));
}

/* lnf (Rust f32::ln): m in [sqrt(2)/2, sqrt(2)), ln m = 2 atanh(f/(2+f)). */
RTW_HD float rtw_logf(float x) {
    if (x != x) return x;
    if (x < 0.0f) return rtw_u2f(0x7FC00000u);
    if (x == 0.0f) return rtw_u2f(0xFF800000u);
    if (x == rtw_u2f(0x7F800000u)) return x;
    const double d = (double)x; /* every f32 (subnormals included) is a normal f64 */
    const uint64_t u = rtw_d2u(d);
    int e = (int)((u >> 52) & 0x7FF) - 1023;
    double m = rtw_u2d((u & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
    if (m > 1.4142135623730951) {
        m = m * 0.5;
        e += 1;
    }
    const double f = m - 1.0;
    const double s = f / (2.0 + f);
    const double s2 = s * s;
    /* 2*(s + s^3/3 + ... + s^25/25); |s| <= 0.1716 -> truncation < 1e-20 */
    double p = 1.0 / 25.0;
    p = p * s2 + 1.0 / 23.0;
    p = p * s2 + 1.0 / 21.0;
    p = p * s2 + 1.0 / 19.0;
    p = p * s2 + 1.0 / 17.0;
    p = p * s2 + 1.0 / 15.0;
    p = p * s2 + 1.0 / 13.0;
    p = p * s2 + 1.0 / 11.0;
    p = p * s2 + 1.0 / 9.0;
    p = p * s2 + 1.0 / 7.0;
    p = p * s2 + 1.0 / 5.0;
    p = p * s2 + 1.0 / 3.0;
    const double lm = 2.0 * (s + s * s2 * p);
    return (float)((double)e * RTW_LN2_D + lm);
}

/* sinf: Cody-Waite reduction by pi/2 in f64 (exact for |x| < 2^20 * pi/2), Taylor kernels. */
RTW_HD double rtw_sin_kernel_d(double r) {
    /* sin r = sum_{k>=0} (-1)^k r^(2k+1)/(2k+1)!, k = 0..9; |r| <= pi/4 -> truncation < 1e-19 */
    const double r2 = r * r;
    const double c9 = -1.0 / 121645100408832000.0;
    const double c8 = 1.0 / 355687428096000.0;
    const double c7 = -1.0 / 1307674368000.0;
    const double c6 = 1.0 / 6227020800.0;
    const double c5 = -1.0 / 39916800.0;
    const double c4 = 1.0 / 362880.0;
    const double c3 = -1.0 / 5040.0;
    const double c2 = 1.0 / 120.0;
    const double c1 = -1.0 / 6.0;
    double t = c9;
    t = t * r2 + c8;
    t = t * r2 + c7;
    t = t * r2 + c6;
    t = t * r2 + c5;
    t = t * r2 + c4;
    t = t * r2 + c3;
    t = t * r2 + c2;
    t = t * r2 + c1;
    return r + r * r2 * t;
}
RTW_HD double rtw_cos_kernel_d(double r) {
    const double r2 = r * r;
    /* cos r = sum_{k>=0} (-1)^k r^(2k)/(2k)!, k = 0..10 */
    const double c10 = 1.0 / 2432902008176640000.0;
    const double c9 = -1.0 / 6402373705728000.0;
    const double c8 = 1.0 / 20922789888000.0;
    const double c7 = -1.0 / 87178291200.0;
    const double c6 = 1.0 / 479001600.0;
    const double c5 = -1.0 / 3628800.0;
    const double c4 = 1.0 / 40320.0;
    const double c3 = -1.0 / 720.0;
    const double c2 = 1.0 / 24.0;
    const double c1 = -1.0 / 2.0;
    double t = c10;
    t = t * r2 + c9;
    t = t * r2 + c8;
    t = t * r2 + c7;
    t = t * r2 + c6;
    t = t * r2 + c5;
    t = t * r2 + c4;
    t = t * r2 + c3;
    t = t * r2 + c2;
    t = t * r2 + c1;
    return 1.0 + r2 * t;
}
RTW_HD float rtw_sinf(float x) {
    if (x != x) return x;
    if (x == rtw_u2f(0x7F800000u) || x == rtw_u2f(0xFF800000u)) return rtw_u2f(0x7FC00000u);
    if (x == 0.0f) return x; /* keeps the sign of zero */
    const double d = (double)x;
    /* k = round(d * 2/pi) */
    const double kd = __builtin_rint(d * 0.63661977236758138243);
    /* pi/2 split into three parts; PIO2_1 has 33 significant bits (k*PIO2_1 exact for |k|<2^20) */
    const double PIO2_1 = 1.57079632673412561417e+00; /* 0x3FF921FB54400000 */
    const double PIO2_2 = 6.07710050630396597660e-11; /* 0x3DD0B4611A600000 */
    const double PIO2_3 = 2.02226624871116645580e-21; /* 0x3BA3198A2E000000 */
    const double r = ((d - kd * PIO2_1) - kd * PIO2_2) - kd * PIO2_3;
    const int64_t k = (int64_t)kd;
    double v;
    switch ((int)(k & 3)) {
        case 0: v = rtw_sin_kernel_d(r); break;
        case 1: v = rtw_cos_kernel_d(r); break;
        case 2: v = -rtw_sin_kernel_d(r); break;
        default: v = -rtw_cos_kernel_d(r); break;
    }
    return (float)v;
}


/* ------------------------------------------------------------------------------------------ */
/* Proximity cull (ours, not in the reference): an extra per-node test ANDed with the          */
/* reference's Aabb::hit_cond.  It never rejects a node below which a cullable leaf's test     */
/* would accept a root in [ts, te), so the closest hit, its tie-breaking and every RNG draw     */
/* are those of the reference traversal (argument and error bounds: DESIGN.md "Proximity       */
/* cull"; node constants k, m: rtw_cull.h).                                                     */
/*   per (ray, node): Dq = sum_i max(|min_i - o_i|, |max_i - o_i|)^2 >= |o - x|^2 for every x  */
/*   in the box, D = sum of the same maxima >= |o - x|; delta = k Dq + 64u D + m bounds how far   */
/*   outside the box a computed hit point of                                                     */
/*   a leaf below can lie (plus the quotient roundings); the node passes when the ray segment   */
/*   [ts, te] meets the box grown by delta, reusing hit_cond's slab quotients.                  */
/* ------------------------------------------------------------------------------------------ */
#define RTW_CULL_U 0x1p-24f
/* delta = k Dq + 64u D + m for a node box and a ray origin, with a_i = min_i - o_i,
 * b_i = max_i - o_i, M_i = max(|a_i|, |b_i|) (the farthest corner's offsets), Dq = sum_i M_i^2 and
 * D = sum_i M_i: for every x in the box |o - x|^2 <= Dq and |o - x| <= D, which is all the bound
 * uses of them.  Fused steps: host and device round identically (any rounding of this bound is far
 * inside the safety factor of the cull analysis). */
RTW_HD float rtw_cull_delta(float k, float m, float a0, float b0, float a1, float b1, float a2, float b2) {
    const float m0 = __builtin_fmaxf(__builtin_fabsf(a0), __builtin_fabsf(b0));
    const float m1 = __builtin_fmaxf(__builtin_fabsf(a1), __builtin_fabsf(b1));
    const float m2 = __builtin_fmaxf(__builtin_fabsf(a2), __builtin_fabsf(b2));
    const float d = (m0 + m1) + m2;
    const float dq = __builtin_fmaf(m2, m2, __builtin_fmaf(m1, m1, m0 * m0));
    return __builtin_fmaf(k, dq, __builtin_fmaf(64.0f * RTW_CULL_U, d, m));
}
/* one axis: [t0 - w, t1 + w] narrows [lo, hi]; NaN operands are dropped (conservative) */
RTW_HD void rtw_cull_axis(float t0, float t1, float w, float* lo, float* hi) {
    *lo = __builtin_fmaxf(*lo, t0 - w);
    *hi = __builtin_fminf(*hi, t1 + w);
}

#ifdef __cplusplus
}
#endif

#endif /* RTW_SCALAR_H */
