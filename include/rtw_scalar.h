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
 *      `texture.rs:32,50`).  The reference calls the platform libm; these restate glibc 2.35's
 *      acosf / atan2f / sinf / logf (the FMA builds x86-64 selects) bit for bit, pinned
 *      exhaustively against the live libm (tests/test_libm.py).
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
 * [0, spp).  The image is therefore independent of lane/thread/GPU assignment.
 * The xoroshiro state is s0 = x = splitmix64's finalizer of (pixel, sample) ^ key, s1 a second,
 * bijective xorshift-multiply round of x (the finalizer's avalanche makes streams of neighbouring
 * pixels and samples independent).  Round 5: one finalizer per sample instead of three (their 64-bit
 * multiplies were most of the kernel's per-sample stream setup); the ctr-vs-ref statistical check
 * (tests/test_ref_mode.py) pins the streams' quality. */
RTW_HD uint64_t rtw_seed_key(uint64_t seed) { return rtw_mix64(seed ^ 0x5EED5EED5EED5EEDull); }
RTW_HD rtw_xoro rtw_sample_stream(uint64_t seed_key, uint32_t pixel, uint32_t sample) {
    const uint64_t x = rtw_mix64((((uint64_t)pixel) << 32 | (uint64_t)sample) ^ seed_key);
    rtw_xoro r;
    r.s0 = x;
    r.s1 = (x ^ (x >> 32)) * 0xD6E8FEB86659FD93ull;
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
/* f32 elementary functions: glibc 2.35's libm, restated bit for bit                          */
/* ------------------------------------------------------------------------------------------ */
/* The reference calls f32::acos / atan2 (vec3.rs:242-243, every sphere uv), f32::sin
 * (texture.rs:32 checker, :50 marble) and f32::ln (hittable.rs:328, volume distance).  On Linux
 * Rust lowers them to the platform libm's acosf / atan2f / sinf / logf.  The platform here is
 * glibc 2.35 (Ubuntu 22.04, this image and the GPU box), x86-64 with FMA, where the dynamic
 * linker's ifunc picks the FMA builds of sinf and logf.  None of the four is correctly rounded
 * (acosf differs from RN(acos) on ~8 % of [-1, 1], atan2f on ~16 %), so the restatement follows
 * glibc's own algorithms and operation order:
 *   acosf   sysdeps/ieee754/flt-32/e_acosf.c   (fdlibm, f32 arithmetic)
 *   atan2f  sysdeps/ieee754/flt-32/e_atan2f.c  (fdlibm) + s_atanf.c
 *   sinf    sysdeps/ieee754/flt-32/s_sinf.c + sincosf.h + sincosf_data.c  (f64 kernels, FMA build)
 *   logf    sysdeps/ieee754/flt-32/e_logf.c + e_logf_data.c             (f64 kernel, FMA build)
 * The FMA builds contract specific multiply-adds; each rtw_fma below marks one of them.  Pinned
 * exhaustively against the live libm (tests/native/libm_check.c: every f32 input of acosf, sinf
 * and logf, 2^28 atan2f pairs; 0 mismatches) and by tests/golden/libm_f32.npz.
 *
 * Notices of the restated algorithms (their coefficients and operation order are reproduced below):
 *
 *   rtw_acosf, rtw_atan2f (e_acosf.c, e_atan2f.c, s_atanf.c; fdlibm, converted to float by Ian Lance
 *   Taylor, Cygnus Support):
 *     Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
 *     Developed at SunPro, a Sun Microsystems, Inc. business.
 *     Permission to use, copy, modify, and distribute this software is freely granted, provided that
 *     this notice is preserved.
 *
 *   rtw_sinf, rtw_logf (s_sinf.c, sincosf.h, sincosf_data.c, e_logf.c, e_logf_data.c): written by
 *   Szabolcs Nagy and others for Arm's optimized-routines (Copyright (c) 2017-2018, Arm Limited;
 *   SPDX-License-Identifier: MIT) and contributed to the GNU C Library (Copyright (C) 2017-2022 Free
 *   Software Foundation, Inc.; the GNU C Library is free software, distributed under the GNU Lesser
 *   General Public License, version 2.1 or any later version). */
RTW_HD double rtw_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

/* e_acosf.c __ieee754_acosf */
RTW_HD float rtw_acosf(float x) {
    const float one = 1.0f, half = 0.5f;
    const float pi = rtw_u2f(0x40490fdau), pio2_hi = rtw_u2f(0x3fc90fdau), pio2_lo = rtw_u2f(0x33a22168u);
    const float pS0 = rtw_u2f(0x3e2aaaabu), pS1 = rtw_u2f(0xbea6b090u), pS2 = rtw_u2f(0x3e4e0aa8u),
                pS3 = rtw_u2f(0xbd241146u), pS4 = rtw_u2f(0x3a4f7f04u), pS5 = rtw_u2f(0x3811ef08u);
    const float qS1 = rtw_u2f(0xc019d139u), qS2 = rtw_u2f(0x4001572du), qS3 = rtw_u2f(0xbf303361u),
                qS4 = rtw_u2f(0x3d9dc62eu);
    const int32_t hx = (int32_t)rtw_f2u(x);
    const int32_t ix = hx & 0x7fffffff;
    float z, p, q, r, w, s;
    if (ix == 0x3f800000) {                               /* |x| == 1 */
        if (hx > 0) return 0.0f;
        return pi + rtw_u2f(0x34222168u);                 /* pi + 2 pio2_lo */
    }
    if (ix > 0x3f800000) return (x - x) / (x - x);        /* |x| > 1 or NaN */
    if (ix < 0x3f000000) {                                /* |x| < 0.5 */
        if (ix <= 0x32800000) return pio2_hi + pio2_lo;   /* |x| <= 2^-26 */
        z = x * x;
        p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        r = p / q;
        return pio2_hi - (x - (pio2_lo - x * r));
    } else if (hx < 0) {                                  /* x < -0.5 */
        z = (one + x) * half;
        p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        s = __builtin_sqrtf(z);
        r = p / q;
        w = r * s - pio2_lo;
        return pi - 2.0f * (s + w);
    } else {                                              /* x > 0.5 */
        z = (one - x) * half;
        s = __builtin_sqrtf(z);
        const float df = rtw_u2f(rtw_f2u(s) & 0xfffff000u);
        const float c = (z - df * df) / (s + df);
        p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        r = p / q;
        w = r * s + c;
        return 2.0f * (df + w);
    }
}

/* s_atanf.c __atanf */
RTW_HD float rtw_atanf(float x) {
    const float one = 1.0f;
    const float atanhi[4] = {rtw_u2f(0x3eed6338u), rtw_u2f(0x3f490fdau), rtw_u2f(0x3f7b985eu), rtw_u2f(0x3fc90fdau)};
    const float atanlo[4] = {rtw_u2f(0x31ac3769u), rtw_u2f(0x33222168u), rtw_u2f(0x33140fb4u), rtw_u2f(0x33a22168u)};
    const float aT0 = rtw_u2f(0x3eaaaaabu), aT1 = rtw_u2f(0xbe4ccccdu), aT2 = rtw_u2f(0x3e124925u),
                aT3 = rtw_u2f(0xbde38e38u), aT4 = rtw_u2f(0x3dba2e6eu), aT5 = rtw_u2f(0xbd9d8795u),
                aT6 = rtw_u2f(0x3d886b35u), aT7 = rtw_u2f(0xbd6ef16bu), aT8 = rtw_u2f(0x3d4bda59u),
                aT9 = rtw_u2f(0xbd15a221u), aT10 = rtw_u2f(0x3c8569d7u);
    const int32_t hx = (int32_t)rtw_f2u(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {                               /* |x| >= 2^25 */
        if (ix > 0x7f800000) return x + x;                /* NaN */
        if (hx > 0) return atanhi[3] + atanlo[3];
        return -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {                                /* |x| < 0.4375 */
        if (ix < 0x31000000) return x;                    /* |x| < 2^-29 */
        id = -1;
    } else {
        x = __builtin_fabsf(x);
        if (ix < 0x3f980000) {                            /* |x| < 1.1875 */
            if (ix < 0x3f300000) {                        /* 7/16 <= |x| < 11/16 */
                id = 0;
                x = (2.0f * x - one) / (2.0f + x);
            } else {                                      /* 11/16 <= |x| < 19/16 */
                id = 1;
                x = (x - one) / (x + one);
            }
        } else if (ix < 0x401c0000) {                     /* |x| < 2.4375 */
            id = 2;
            x = (x - 1.5f) / (one + 1.5f * x);
        } else {                                          /* 2.4375 <= |x| < 2^25 */
            id = 3;
            x = -1.0f / x;
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return (hx < 0) ? -r : r;
}

/* e_atan2f.c __ieee754_atan2f (the w_atan2f wrapper only sets errno) */
RTW_HD float rtw_atan2f(float y, float x) {
    const float tiny = rtw_u2f(0x0da24260u);              /* 1.0e-30 */
    const float pi_o_4 = rtw_u2f(0x3f490fdbu), pi_o_2 = rtw_u2f(0x3fc90fdbu), pi = rtw_u2f(0x40490fdbu),
                pi_lo = rtw_u2f(0xb3bbbd2eu);
    const int32_t hx = (int32_t)rtw_f2u(x), hy = (int32_t)rtw_f2u(y);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y; /* NaN */
    if (hx == 0x3f800000) return rtw_atanf(y);            /* x = 1 */
    const int m = (int)(((uint32_t)hy >> 31) & 1u) | (int)(((uint32_t)hx >> 30) & 2u);
    if (iy == 0) {
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (ix == 0) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;                /* |y/x| > 2^60 */
    else if (hx < 0 && k < -60) z = 0.0f;                 /* |y|/x < -2^60 */
    else z = rtw_atanf(__builtin_fabsf(y / x));
    switch (m) {
        case 0: return z;
        case 1: return rtw_u2f(rtw_f2u(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

/* e_logf.c __logf with e_logf_data.c (LOGF_TABLE_BITS 4, poly order 4); FMA build. */
RTW_HD float rtw_logf(float x) {
    /* {invc, logc}: 1/c and log(c) for the 16 subintervals of [0x3f330000, 2 * 0x3f330000) */
    const uint64_t T[16][2] = {
        {0x3ff661ec79f8f3beull, 0xbfd57bf7808caadeull}, {0x3ff571ed4aaf883dull, 0xbfd2bef0a7c06ddbull},
        {0x3ff49539f0f010b0ull, 0xbfd01eae7f513a67ull}, {0x3ff3c995b0b80385ull, 0xbfcb31d8a68224e9ull},
        {0x3ff30d190c8864a5ull, 0xbfc6574f0ac07758ull}, {0x3ff25e227b0b8ea0ull, 0xbfc1aa2bc79c8100ull},
        {0x3ff1bb4a4a1a343full, 0xbfba4e76ce8c0e5eull}, {0x3ff12358f08ae5baull, 0xbfb1973c5a611cccull},
        {0x3ff0953f419900a7ull, 0xbfa252f438e10c1eull}, {0x3ff0000000000000ull, 0x0000000000000000ull},
        {0x3fee608cfd9a47acull, 0x3faaa5aa5df25984ull}, {0x3feca4b31f026aa0ull, 0x3fbc5e53aa362eb4ull},
        {0x3feb2036576afce6ull, 0x3fc526e57720db08ull}, {0x3fe9c2d163a1aa2dull, 0x3fcbc2860d224770ull},
        {0x3fe886e6037841edull, 0x3fd1058bc8a07ee1ull}, {0x3fe767dcf5534862ull, 0x3fd4043057b6ee09ull}};
    const double Ln2 = rtw_u2d(0x3fe62e42fefa39efull);
    const double A0 = rtw_u2d(0xbfd00ea348b88334ull), A1 = rtw_u2d(0x3fd5575b0be00b6aull),
                 A2 = rtw_u2d(0xbfdffffef20a4123ull);
    uint32_t ix = rtw_f2u(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) { /* subnormal, zero, negative, inf, NaN */
        if (ix * 2u == 0u) return rtw_u2f(0xff800000u);    /* -inf (divide by zero) */
        if (ix == 0x7f800000u) return x;                  /* log(inf) = inf */
        if ((ix & 0x80000000u) || ix * 2u >= 0xff000000u) return (x - x) / (x - x);
        ix = rtw_f2u(x * 0x1p23f);                        /* subnormal: normalise */
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) % 16u);
    const int32_t k = (int32_t)tmp >> 23;                 /* arithmetic shift */
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const double invc = rtw_u2d(T[i][0]), logc = rtw_u2d(T[i][1]);
    const double z = (double)rtw_u2f(iz);
    const double r = rtw_fma(z, invc, -1.0);              /* z * invc - 1 */
    const double y0 = rtw_fma((double)k, Ln2, logc);      /* logc + k * Ln2 */
    const double r2 = r * r;
    double y = rtw_fma(A1, r, A2);                        /* A[1] * r + A[2] */
    y = rtw_fma(A0, r2, y);                               /* A[0] * r2 + y */
    y = rtw_fma(y, r2, y0 + r);                           /* y * r2 + (y0 + r) */
    return (float)y;
}

/* sincosf_data.c __sincosf_table[0] (quadrants 0, 1) and [1] (2, 3): the sine coefficients are
 * shared, the cosine ones negated in [1].  {c0, c1, s1, c2, s2, c3, s3, c4}. */
RTW_HD double rtw_sincosf_coef(int table, int j) {
    const uint64_t C[2][8] = {
        {0x3ff0000000000000ull, 0xbfdffffffd0c621cull, 0xbfc555545995a603ull, 0x3fa55553e1068f19ull,
         0x3f81107605230bc4ull, 0xbf56c087e89a359dull, 0xbf2994eb3774cf24ull, 0x3ef99343027bf8c3ull},
        {0xbff0000000000000ull, 0x3fdffffffd0c621cull, 0xbfc555545995a603ull, 0xbfa55553e1068f19ull,
         0x3f81107605230bc4ull, 0x3f56c087e89a359dull, 0xbf2994eb3774cf24ull, 0xbef99343027bf8c3ull}};
    return rtw_u2d(C[table][j]);
}
/* sincosf.h sinf_poly: n even -> sine polynomial of x (x2 = x*x of the unsigned remainder),
 * n odd -> cosine polynomial; FMA build. */
RTW_HD float rtw_sinf_poly(double x, double x2, int table, int n) {
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = rtw_fma(x2, rtw_sincosf_coef(table, 6), rtw_sincosf_coef(table, 4)); /* s2 + x2 s3 */
        const double x7 = x3 * x2;
        const double s = rtw_fma(x3, rtw_sincosf_coef(table, 2), x);                            /* x + x3 s1 */
        return (float)rtw_fma(x7, s1, s);
    }
    const double x4 = x2 * x2;
    const double c2 = rtw_fma(x2, rtw_sincosf_coef(table, 7), rtw_sincosf_coef(table, 5));     /* c3 + x2 c4 */
    const double c1 = rtw_fma(x2, rtw_sincosf_coef(table, 1), rtw_sincosf_coef(table, 0));     /* c0 + x2 c1 */
    const double x6 = x4 * x2;
    const double c = rtw_fma(x4, rtw_sincosf_coef(table, 3), c1);                               /* c1 + x4 c2 */
    return (float)rtw_fma(x6, c2, c);
}
/* sincosf.h reduce_large: x * 4/pi in 2.62 fixed point from __inv_pio4 (the bits of 4/pi),
 * for 120 <= |x| < inf; returns the remainder in radians, n = the quadrant. */
RTW_HD double rtw_sinf_reduce_large(uint32_t xi, int* np) {
    const uint32_t inv_pio4[24] = {
        0xa2u, 0xa2f9u, 0xa2f983u, 0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u, 0x6e4e4415u, 0x4e441529u,
        0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u, 0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u,
        0x34ddc0dbu, 0xddc0db62u, 0xc0db6295u, 0xdb629599u, 0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u};
    const uint32_t* arr = &inv_pio4[(xi >> 26) & 15u];
    const int shift = (int)((xi >> 23) & 7u);
    xi = (xi & 0xffffffu) | 0x800000u;
    xi <<= shift;
    uint64_t res0 = (uint64_t)(uint32_t)(xi * arr[0]);
    const uint64_t res1 = (uint64_t)xi * arr[4];
    const uint64_t res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ull << 61)) >> 62;
    res0 -= n << 62;
    *np = (int)n;
    return (double)(int64_t)res0 * rtw_u2d(0x3c1921fb54442d18ull); /* pi / 2^63 */
}
/* s_sinf.c sinf; FMA build. */
RTW_HD float rtw_sinf(float y) {
    const double sign[4] = {1.0, -1.0, -1.0, 1.0};
    double x = (double)y;
    const uint32_t top = (rtw_f2u(y) >> 20) & 0x7ffu;
    if (top < 0x3f4u) {                                   /* |y| < pi/4 */
        if (top < 0x398u) return y;                       /* |y| < 2^-12 */
        return rtw_sinf_poly(x, x * x, 0, 0);
    }
    if (top < 0x42fu) {                                   /* |y| < 120: reduce_fast */
        const double r = x * rtw_u2d(0x41645f306dc9c883ull);     /* x * 2/pi * 2^24 */
        const int n = ((int32_t)r + 0x800000) >> 24;
        x = rtw_fma(-(double)n, rtw_u2d(0x3ff921fb54442d18ull), x); /* x - n pi/2 */
        return rtw_sinf_poly(x * sign[n & 3], x * x, (n & 2) ? 1 : 0, n);
    }
    if (top < 0x7f8u) {                                   /* finite */
        const uint32_t xi = rtw_f2u(y);
        const int s = (int)(xi >> 31);
        int n;
        x = rtw_sinf_reduce_large(xi, &n);
        return rtw_sinf_poly(x * sign[(n + s) & 3], x * x, ((n + s) & 2) ? 1 : 0, n);
    }
    return (y - y) / (y - y);                             /* inf, NaN */
}

/* CheckerTexture reads only the sign of RN(RN(sin x sin y) sin z) (texture.rs:32-33).  The sign
 * of one sine follows from a Cody-Waite reduction x = k pi/2 + r (three-part pi/2, exact for
 * |x| < 2^19) whenever |r| > 2^-30: sin x then has the sign of sin r, cos r > 0, -sin r or -cos r
 * for k = 0, 1, 2, 3 mod 4, and |sin x| > 2^-31, so glibc's sinf (error < 1 ulp) has that sign and
 * none of the two f32 products is zero or subnormal.  Returns 1 and sets *neg when decided, 0 when
 * the sine must be evaluated (0, |x| >= 2^19, NaN, x next to a multiple of pi/2).  Pinned against
 * the live libm's sinf sign for every f32 (tests/native/libm_check.c mode sinsign). */
RTW_HD int rtw_sin_sign_fast(float x, int* neg) {
    const double d = __builtin_fabs((double)x) < 0x1p19 ? (double)x : 0.0; /* NaN, huge -> 0 */
    const double kd = __builtin_rint(d * 0.63661977236758138243);
    const double r = ((d - kd * 1.57079632673412561417e+00) - kd * 6.07710050630396597660e-11) -
                     kd * 2.02226624871116645580e-21;
    const int q = (int)kd & 3;
    *neg = (q == 0) ? r < 0.0 : (q == 2) ? r > 0.0 : q == 3;
    return __builtin_fabs(r) > 0x1p-30;                   /* d = 0 (also 0, NaN, huge x): undecided */
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
