/* TEST INFRASTRUCTURE: pins the f32 elementary functions of include/rtw_scalar.h against the live
 * platform libm (glibc 2.35 here and on the GPU box), which is what the reference's f32::acos /
 * atan2 / sin / ln call (vec3.rs:242-243, texture.rs:32,50, hittable.rs:328).
 *
 *   libm_check <mode> <threads> [lo hi]      modes: acosf sinf logf  (f32 bit patterns [lo, hi),
 *                                                    default all 2^32)
 *                                                   sinsign  (rtw_sin_sign_fast vs sign of sinf)
 *   libm_check atan2f <threads> <pairs>      random pairs (bit patterns, [-2,2]^2, close
 *                                             magnitudes, unit-normal components) + a special grid
 * Prints "mode=... tested=N mismatches=M"; exit status 1 on any mismatch.  NaN equals NaN (any
 * payload: the render path only casts or compares them). */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/rtw_scalar.h"

static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline int same(float a, float b) { return (a != a && b != b) || f2u(a) == f2u(b); }

typedef struct {
    int mode, tid, nthreads;
    uint64_t lo, hi, pairs;
    uint64_t tested, bad, undecided;
    float ex[3];
} job_t;

enum { M_ACOS, M_SIN, M_LOG, M_SINSIGN, M_ATAN2 };

static void report(job_t* j, float a, float b, float got, float want) {
    if (j->bad < 4) printf("MISMATCH mode=%d x=%a (0x%08x) y=%a got=%a want=%a\n", j->mode, a, f2u(a), b, got, want);
    ++j->bad;
}

static inline uint64_t xs(uint64_t* s) {
    uint64_t x = *s;
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    return *s = x;
}

static void check_atan2(job_t* j, float y, float x) {
    const float got = rtw_atan2f(y, x), want = atan2f(y, x);
    ++j->tested;
    if (!same(got, want)) report(j, y, x, got, want);
}

static void* run(void* arg) {
    job_t* j = (job_t*)arg;
    if (j->mode == M_ATAN2) {
        uint64_t s = 0x9E3779B97F4A7C15ull ^ ((uint64_t)(j->tid + 1) * 0xD1B54A32D192ED03ull);
        for (uint64_t i = (uint64_t)j->tid; i < j->pairs; i += (uint64_t)j->nthreads) {
            const uint64_t r = xs(&s);
            float y, x;
            switch (i & 3) {
                case 0: y = u2f((uint32_t)r); x = u2f((uint32_t)(r >> 32)); break;
                case 1: /* uniform in [-2, 2]^2 */
                    y = (float)((double)(uint32_t)r / 4294967296.0 * 4.0 - 2.0);
                    x = (float)((double)(uint32_t)(r >> 32) / 4294967296.0 * 4.0 - 2.0);
                    break;
                case 2: { /* close magnitudes, any exponent: every atanf reduction branch */
                    const uint32_t e = (uint32_t)(r % 254u) + 1u;
                    const uint32_t ya = (e << 23) | ((uint32_t)(r >> 8) & 0x7FFFFFu);
                    const int32_t dx = (int32_t)((r >> 32) & 0x1FFFFFFu) - 0x1000000;
                    uint32_t xa = (uint32_t)((int32_t)ya + dx * ((r >> 60) & 1u ? 1 : 16));
                    if (xa >= 0x7F800000u) xa = ya;
                    y = u2f(ya | ((uint32_t)(r >> 61) & 1u) << 31);
                    x = u2f(xa | ((uint32_t)(r >> 62) & 1u) << 31);
                    break;
                }
                default: { /* sphere uv: atan2(-z, x) of a unit normal */
                    const double a = (double)(uint32_t)r / 4294967296.0 * 6.283185307179586;
                    const double c = (double)(uint32_t)(r >> 32) / 4294967296.0 * 2.0 - 1.0;
                    const double q = sqrt(1.0 - c * c);
                    y = (float)(-q * sin(a));
                    x = (float)(q * cos(a));
                    break;
                }
            }
            check_atan2(j, y, x);
        }
        if (j->tid == 0) { /* special values and exact ratios */
            const float sp[] = {0.0f, -0.0f, 1.0f, -1.0f, INFINITY, -INFINITY, NAN, 1e-45f, -1e-45f, 3.4e38f,
                                -3.4e38f, 0.5f, 2.0f, 0x1p-60f, 0x1p60f, 0x1p-100f, 0x1p100f, 1.1754944e-38f};
            const int n = (int)(sizeof sp / sizeof sp[0]);
            for (int a = 0; a < n; ++a)
                for (int b = 0; b < n; ++b) check_atan2(j, sp[a], sp[b]);
        }
        return NULL;
    }
    for (uint64_t u = j->lo + (uint64_t)j->tid; u < j->hi; u += (uint64_t)j->nthreads) {
        const float x = u2f((uint32_t)u);
        ++j->tested;
        if (j->mode == M_SINSIGN) {
            int neg;
            if (!rtw_sin_sign_fast(x, &neg)) { ++j->undecided; continue; }
            const float s = sinf(x);
            if (!(s != 0.0f && s == s) || (s < 0.0f) != (neg != 0) || fabsf(s) <= 0x1p-31f) report(j, x, 0, (float)neg, s);
            continue;
        }
        float got, want;
        switch (j->mode) {
            case M_ACOS: got = rtw_acosf(x); want = acosf(x); break;
            case M_SIN: got = rtw_sinf(x); want = sinf(x); break;
            default: got = rtw_logf(x); want = logf(x); break;
        }
        if (!same(got, want)) report(j, x, 0, got, want);
    }
    return NULL;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s acosf|sinf|logf|sinsign|atan2f threads [lo hi | pairs]\n", argv[0]);
        return 2;
    }
    const char* m = argv[1];
    const int mode = !strcmp(m, "acosf") ? M_ACOS : !strcmp(m, "sinf") ? M_SIN : !strcmp(m, "logf") ? M_LOG
                   : !strcmp(m, "sinsign") ? M_SINSIGN : !strcmp(m, "atan2f") ? M_ATAN2 : -1;
    if (mode < 0) return 2;
    int nt = atoi(argv[2]);
    if (nt < 1) nt = 1;
    if (nt > 256) nt = 256;
    uint64_t lo = 0, hi = 1ull << 32, pairs = 1ull << 28;
    if (mode == M_ATAN2 && argc > 3) pairs = strtoull(argv[3], NULL, 0);
    if (mode != M_ATAN2 && argc > 4) { lo = strtoull(argv[3], NULL, 0); hi = strtoull(argv[4], NULL, 0); }
    job_t* jobs = calloc((size_t)nt, sizeof(job_t));
    pthread_t* th = calloc((size_t)nt, sizeof(pthread_t));
    for (int t = 0; t < nt; ++t) {
        jobs[t] = (job_t){.mode = mode, .tid = t, .nthreads = nt, .lo = lo, .hi = hi, .pairs = pairs};
        pthread_create(&th[t], NULL, run, &jobs[t]);
    }
    uint64_t tested = 0, bad = 0, und = 0;
    for (int t = 0; t < nt; ++t) {
        pthread_join(th[t], NULL);
        tested += jobs[t].tested;
        bad += jobs[t].bad;
        und += jobs[t].undecided;
    }
    printf("mode=%s tested=%llu undecided=%llu mismatches=%llu\n", m, (unsigned long long)tested,
           (unsigned long long)und, (unsigned long long)bad);
    return bad ? 1 : 0;
}
