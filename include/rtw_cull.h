/*
 * rtw_cull.h -- upload-time constants of the proximity cull (rtw_scalar.h rtw_cull_*,
 * DESIGN.md "Proximity cull"), shared by librtw.so and the oracle's culled mode so both
 * evaluate the identical per-node test.  Host-only C99/C++.
 *
 * km[2 n] = k, km[2 n + 1] = m for node n; the per-(ray, node) margin is
 *   delta = k D^2 + 64u D + m      (u = 2^-24, D = sum_i |min_i - o_i| + |max_i - o_i|)
 * k and m are the maxima over the leaves below n of
 *   plain sphere (SurfaceGeometry, no Transformation/Animation, hittable.rs:212-247; sphere
 *     test sphere_geometry.rs:21-59):  k = 64u / r,  m = 8u (max_i |c_i| + r)
 *   plain triangle (triangle_geometry.rs:13-45):  k = 0,  m = u (16 A + 64 kappa diam)
 *     A = max |p_ji|, diam = longest edge, kappa = max_{edges e != f} |e| |f| / |e x f| (>= 1/sin
 *     of the smallest angle); a triangle whose f32 cross product is zero can never hit (its
 *     normal is NaN) and adds nothing.
 * and k = +inf (never culled) when any other leaf is below (rects, boxes, volumes, transformed
 * or animated leaves: their hit points are not bounded by the culled box -- the reference's
 * apply_aabb quirk), when kappa > 2^16, or when a leaf's own Aabb (aabb.rs new_radius /
 * new_surrounding_points) is not inside the node box.
 * tests/native/cull_bound_check.c stresses the bound: every accepted sphere/triangle hit passes.
 */
#ifndef RTW_CULL_H
#define RTW_CULL_H

#include <math.h>

#include "rtw.h"
#include "rtw_scalar.h"

typedef struct rtw_cull_acc {
    float k, m, lo[3], hi[3];
    int ok;
} rtw_cull_acc;

static void rtw_cull_acc_init(rtw_cull_acc* a) {
    const float inf = rtw_u2f(0x7F800000u);
    a->k = 0.0f;
    a->m = 0.0f;
    for (int i = 0; i < 3; ++i) { a->lo[i] = inf; a->hi[i] = -inf; }
    a->ok = 1;
}

static void rtw_cull_acc_box(rtw_cull_acc* a, const float lo[3], const float hi[3]) {
    for (int i = 0; i < 3; ++i) {
        if (lo[i] < a->lo[i]) a->lo[i] = lo[i];
        if (hi[i] > a->hi[i]) a->hi[i] = hi[i];
    }
}

/* One sphere (centre c, radius r): constants and Aabb::new_radius.  0 if not cullable. */
static int rtw_cull_sphere(const float c[3], float r, float* k, float* m, float lo[3], float hi[3]) {
    const float inf = rtw_u2f(0x7F800000u);
    if (!(r > 0.0f && r < inf)) return 0;
    float cm = 0.0f;
    for (int i = 0; i < 3; ++i) {
        const float a = __builtin_fabsf(c[i]);
        if (!(a < inf)) return 0;
        if (a > cm) cm = a;
        lo[i] = c[i] - r;
        hi[i] = c[i] + r;
    }
    *k = (64.0f * RTW_CULL_U) / r;
    *m = (8.0f * RTW_CULL_U) * (cm + r);
    return *k < inf && *m < inf;
}

/* One triangle: constants and Aabb::new_surrounding_points.  0 if not cullable; *never = 1 if
 * it can never report a hit (zero f32 cross product, hence a NaN normal). */
static int rtw_cull_triangle(const float p[3][3], float* k, float* m, float lo[3], float hi[3], int* never) {
    const float inf = rtw_u2f(0x7F800000u);
    *never = 0;
    float A = 0.0f;
    for (int i = 0; i < 3; ++i) {
        lo[i] = p[0][i];
        hi[i] = p[0][i];
        for (int j = 0; j < 3; ++j) {
            const float a = __builtin_fabsf(p[j][i]);
            if (!(a < inf)) return 0;
            if (a > A) A = a;
            if (p[j][i] < lo[i]) lo[i] = p[j][i];
            if (p[j][i] > hi[i]) hi[i] = p[j][i];
        }
    }
    /* the reference's own f32 cross (triangle_geometry.rs:16-18) */
    float e1f[3], e2f[3];
    for (int i = 0; i < 3; ++i) { e1f[i] = p[1][i] - p[0][i]; e2f[i] = p[2][i] - p[0][i]; }
    const float cf0 = e1f[1] * e2f[2] - e1f[2] * e2f[1];
    const float cf1 = e1f[2] * e2f[0] - e1f[0] * e2f[2];
    const float cf2 = e1f[0] * e2f[1] - e1f[1] * e2f[0];
    if (cf0 == 0.0f && cf1 == 0.0f && cf2 == 0.0f) { *never = 1; return 1; }
    /* exact-ish shape factor in double */
    double e[3][3];
    for (int i = 0; i < 3; ++i) {
        e[0][i] = (double)p[1][i] - (double)p[0][i];
        e[1][i] = (double)p[2][i] - (double)p[0][i];
        e[2][i] = (double)p[2][i] - (double)p[1][i];
    }
    const double cx = e[0][1] * e[1][2] - e[0][2] * e[1][1];
    const double cy = e[0][2] * e[1][0] - e[0][0] * e[1][2];
    const double cz = e[0][0] * e[1][1] - e[0][1] * e[1][0];
    const double cl = sqrt(cx * cx + cy * cy + cz * cz);
    double len[3], diam = 0.0;
    for (int j = 0; j < 3; ++j) {
        len[j] = sqrt(e[j][0] * e[j][0] + e[j][1] * e[j][1] + e[j][2] * e[j][2]);
        if (len[j] > diam) diam = len[j];
    }
    if (!(cl > 0.0)) return 0;
    double kappa = len[0] * len[1];
    if (len[0] * len[2] > kappa) kappa = len[0] * len[2];
    if (len[1] * len[2] > kappa) kappa = len[1] * len[2];
    kappa /= cl;
    if (!(kappa <= 65536.0)) return 0;
    const double mm = (double)RTW_CULL_U * (16.0 * (double)A + 64.0 * kappa * diam);
    *k = 0.0f;
    *m = (float)(mm * (1.0 + 0x1p-20)); /* rounded up */
    return *m < inf;
}

static void rtw_cull_visit(const rtw_world* w, int32_t n, int depth, float* km, rtw_cull_acc* acc) {
    const float inf = rtw_u2f(0x7F800000u);
    if (depth > 64) { acc->ok = 0; return; }
    if (n < 0) {
        const int32_t li = -1 - n;
        if (li >= w->leaf_count) { acc->ok = 0; return; }
        const rtw_leaf* L = &w->leaves[li];
        float k = 0.0f, m = 0.0f, lo[3], hi[3];
        int good = 0, never = 0;
        if (L->flags == 0 && L->geom_kind == RTW_GEOM_SPHERE && L->geom_index >= 0 &&
            L->geom_index < w->sphere_count) {
            const rtw_sphere* s = &w->spheres[L->geom_index];
            good = rtw_cull_sphere(s->center, s->radius, &k, &m, lo, hi);
        } else if (L->flags == 0 && L->geom_kind == RTW_GEOM_TRIANGLE && L->geom_index >= 0 &&
                   L->geom_index < w->triangle_count) {
            good = rtw_cull_triangle(w->triangles[L->geom_index].positions, &k, &m, lo, hi, &never);
        }
        if (!good) { acc->ok = 0; return; }
        if (never) return;
        if (k > acc->k) acc->k = k;
        if (m > acc->m) acc->m = m;
        rtw_cull_acc_box(acc, lo, hi);
        return;
    }
    if (n >= w->node_count) { acc->ok = 0; return; }
    const rtw_bvh_node* nd = &w->nodes[n];
    rtw_cull_acc sub;
    rtw_cull_acc_init(&sub);
    rtw_cull_visit(w, nd->left, depth + 1, km, &sub);
    rtw_cull_visit(w, nd->right, depth + 1, km, &sub);
    int inside = 1;
    for (int i = 0; i < 3; ++i)
        if (sub.lo[i] <= sub.hi[i] && !(nd->min[i] <= sub.lo[i] && sub.hi[i] <= nd->max[i])) inside = 0;
    const int cull = sub.ok && inside;
    km[2 * (size_t)n] = cull ? sub.k : inf;
    km[2 * (size_t)n + 1] = cull ? sub.m : inf;
    if (!sub.ok) acc->ok = 0;
    if (sub.k > acc->k) acc->k = sub.k;
    if (sub.m > acc->m) acc->m = sub.m;
    rtw_cull_acc_box(acc, sub.lo, sub.hi);
}

/* km: 2 * node_count floats.  disable != 0: every node gets k = +inf (reference traversal). */
static inline void rtw_cull_prepare(const rtw_world* w, float* km, int disable) {
    const float inf = rtw_u2f(0x7F800000u);
    for (int32_t n = 0; n < w->node_count; ++n) {
        km[2 * (size_t)n] = inf;
        km[2 * (size_t)n + 1] = inf;
    }
    if (disable || w->root < 0) return;
    rtw_cull_acc top;
    rtw_cull_acc_init(&top);
    rtw_cull_visit(w, w->root, 0, km, &top);
}

#endif /* RTW_CULL_H */
