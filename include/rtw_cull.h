/*
 * rtw_cull.h -- upload-time constants of the proximity cull (rtw_scalar.h rtw_cull_*,
 * DESIGN.md "Proximity cull"), shared by librtw.so and the oracle's culled mode so both
 * evaluate the identical per-node test.  Host-only C99/C++.
 *
 * km[2 n] = k, km[2 n + 1] = m for node n; the per-(ray, node) margin is
 *   delta = k Dq + 64u D + m      (u = 2^-24; Dq, D: rtw_cull_delta)
 * k and m are the maxima over the leaves below n of
 *   plain sphere (SurfaceGeometry, no Transformation/Animation, hittable.rs:212-247; sphere
 *     test sphere_geometry.rs:21-59):  k = 64u / r,  m = 8u (max_i |c_i| + r)
 *   plain triangle (triangle_geometry.rs:13-45):  k = 0,  m = u (16 A + 64 kappa diam)
 *     A = max |p_ji|, diam = longest edge, kappa = max_{edges e != f} |e| |f| / |e x f| (>= 1/sin
 *     of the smallest angle); a triangle whose f32 cross product is zero can never hit (its
 *     normal is NaN) and adds nothing.
 *   plain rect (rect_geometry.rs:33-59):  k = 0,  m = 8u max(|dist|, |r0|, |r1|): an accepted point
 *     has its in-plane coordinates inside the rect exactly (the test compares them) and its normal
 *     coordinate within 3u |dist - o_n| + u |pos_n| of the plane (t = RN(RN(dist - o_n) / d_n),
 *     pos = RN(o + RN(t d))); the 3u D part is inside the 64u D term.  Box: the flat rect.
 *   plain box primitive (aabb.rs:80-167):  k = 0,  m = 8u max |corner|: the accepted point lies on
 *     its near / far slab plane and inside the other slabs' rounded quotient intervals, each
 *     within 3u |c - o| + u |pos| of the box.
 *   wrapped leaf (Transformation / Animation, hittable.rs:234-244), for trees built over the true
 *     world bounds (the SAH tree, `wrapped` = 1): the local primitive's k, m plus 16u A_w, A_w =
 *     max(|world bound|, |offset| + |velocity| T), T = max |shutter time|.  The leaf tests the
 *     rounded local ray o' = RN(R^T RN(o - off - RN(v time))), d' = RN(R^T d): the exact world point
 *     o + t d lies within |o' - exact| + t |d' - exact| <= 5u |o - off'| + 3u t |d| of the image of
 *     the local point, i.e. within 8u (D + A_w) more; the 8u D part is inside the 64u D term.  The
 *     box: the local bounds mapped by the exact inverse of the device's float transform, rounded
 *     outward.
 * and k = +inf (never culled) when any other leaf is below (volumes; wrapped leaves in the
 * reference tree, whose boxes hold the reference's own Aabbs, not the geometry -- its apply_aabb
 * quirk), when kappa > 2^16, or when a leaf's box is not inside the node box.
 * tests/native/cull_bound_check.c stresses the bound: every accepted hit of every kind passes.
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

/* (p0, p1, n) of a rect plane (rect_geometry.rs:15-21) */
static void rtw_rect_axes(int32_t plane, int* p0, int* p1, int* n) {
    *p0 = plane == RTW_PLANE_YZ ? 1 : 0;
    *p1 = plane == RTW_PLANE_XY ? 1 : 2;
    *n = plane == RTW_PLANE_XY ? 2 : (plane == RTW_PLANE_XZ ? 1 : 0);
}

/* One rect: constants and its flat box.  0 if not cullable. */
static int rtw_cull_rect(const rtw_rect* r, float* k, float* m, float lo[3], float hi[3]) {
    const float inf = rtw_u2f(0x7F800000u);
    int p0, p1, n;
    if (r->plane < 0 || r->plane > 2) return 0;
    rtw_rect_axes(r->plane, &p0, &p1, &n);
    const float v[5] = {r->dist, r->r0[0], r->r0[1], r->r1[0], r->r1[1]};
    float A = 0.0f;
    for (int i = 0; i < 5; ++i) {
        const float a = __builtin_fabsf(v[i]);
        if (!(a < inf)) return 0;
        if (a > A) A = a;
    }
    lo[n] = hi[n] = r->dist;
    lo[p0] = rtw_minr(r->r0[0], r->r0[1]);
    hi[p0] = rtw_maxr(r->r0[0], r->r0[1]);
    lo[p1] = rtw_minr(r->r1[0], r->r1[1]);
    hi[p1] = rtw_maxr(r->r1[0], r->r1[1]);
    *k = 0.0f;
    *m = (8.0f * RTW_CULL_U) * A;
    return *m < inf;
}

/* One box primitive: constants and the box.  0 if not cullable. */
static int rtw_cull_box(const rtw_box* b, float* k, float* m, float lo[3], float hi[3]) {
    const float inf = rtw_u2f(0x7F800000u);
    float A = 0.0f;
    for (int i = 0; i < 3; ++i) {
        const float a = rtw_maxr(__builtin_fabsf(b->min[i]), __builtin_fabsf(b->max[i]));
        if (!(a < inf) || !(b->min[i] <= b->max[i])) return 0;
        if (a > A) A = a;
        lo[i] = b->min[i];
        hi[i] = b->max[i];
    }
    *k = 0.0f;
    *m = (8.0f * RTW_CULL_U) * A;
    return *m < inf;
}

/* The world box of a wrapped leaf's local box: the device reverses a Transformation with
 * o' = M (o - off), M = [[yc, 0, -ys], [0, 1, 0], [ys, 0, yc]] (rot_up(yc, -ys), hittable.rs:271-277),
 * and an Animation with o' = o - v time, time in [t0, t1] (the camera shutter); the world geometry is
 * off + M^-1 G swept by v [t0, t1].  Corners mapped in double with the exact M^-1; each bound moved
 * out by 2^-40 of the magnitudes summed into it (far above double rounding), then rounded outward to
 * f32.  An exact 0 stays 0. */
static int rtw_wrap_box(const rtw_leaf* L, float t0, float t1, const float llo[3], const float lhi[3], float lo[3],
                        float hi[3]) {
    double dlo[3], dhi[3], mag[3];
    for (int i = 0; i < 3; ++i) {
        dlo[i] = llo[i];
        dhi[i] = lhi[i];
        mag[i] = fmax(fabs((double)llo[i]), fabs((double)lhi[i]));
    }
    if (L->flags & RTW_LEAF_TRANSFORM) {
        const double c = L->y_cos, s = L->y_sin, det = c * c + s * s;
        if (!(det > 0.5 && det < 2.0)) return 0;
        double nlo[3] = {1e300, 1e300, 1e300}, nhi[3] = {-1e300, -1e300, -1e300};
        for (int q = 0; q < 8; ++q) {
            const double x = (q & 1) ? dhi[0] : dlo[0], y = (q & 2) ? dhi[1] : dlo[1], z = (q & 4) ? dhi[2] : dlo[2];
            /* M^-1 = [[c, 0, s], [0, 1, 0], [-s, 0, c]] / det on the xz components */
            const double p[3] = {(c * x + s * z) / det + L->offset[0], y + L->offset[1], (-s * x + c * z) / det + L->offset[2]};
            for (int i = 0; i < 3; ++i) {
                if (p[i] < nlo[i]) nlo[i] = p[i];
                if (p[i] > nhi[i]) nhi[i] = p[i];
            }
        }
        const double mxz = 2.0 * (fabs(c) + fabs(s)) * fmax(mag[0], mag[2]);
        mag[0] = mxz + fabs((double)L->offset[0]);
        mag[1] = mag[1] + fabs((double)L->offset[1]);
        mag[2] = mxz + fabs((double)L->offset[2]);
        for (int i = 0; i < 3; ++i) { dlo[i] = nlo[i]; dhi[i] = nhi[i]; }
    }
    if (L->flags & RTW_LEAF_ANIMATION) {
        for (int i = 0; i < 3; ++i) {
            const double a = (double)L->velocity[i] * t0, b = (double)L->velocity[i] * t1;
            dlo[i] += a < b ? a : b;
            dhi[i] += a < b ? b : a;
            mag[i] += fmax(fabs(a), fabs(b));
        }
    }
    for (int i = 0; i < 3; ++i) {
        const double ml = dlo[i] - mag[i] * 0x1p-40, mh = dhi[i] + mag[i] * 0x1p-40;
        lo[i] = (float)ml;
        hi[i] = (float)mh;
        if ((double)lo[i] > ml) lo[i] = nextafterf(lo[i], -INFINITY);
        if ((double)hi[i] < mh) hi[i] = nextafterf(hi[i], INFINITY);
        if (!(lo[i] > -INFINITY && hi[i] < INFINITY)) return 0;
    }
    return 1;
}

/* The interval every ray's time lies in (camera.rs:186-190): start in [time0, time1] (gen_range, or
 * time0 when equal) plus dot(shutter_pace, (px, py)) at the jittered pixel coordinates px, py in [0, 2]
 * (px = x / (W - 1) <= 1 plus a jitter below 1 / (W - 1) <= 1).  With a non-zero pace the device's f32
 * products and sums round (at most 4u of the magnitudes involved), so the bounds move out by 2^-20 of
 * them; rounded outward to f32.  0 if not finite. */
static int rtw_ray_time_range(const rtw_camera* c, float* lo, float* hi) {
    const double a = c->time0 < c->time1 ? c->time0 : c->time1, b = c->time0 < c->time1 ? c->time1 : c->time0;
    const double p0 = c->shutter_pace[0], p1 = c->shutter_pace[1];
    if (!(fabs(a) < 1e300 && fabs(b) < 1e300 && fabs(p0) < 1e300 && fabs(p1) < 1e300)) return 0;
    if (p0 == 0.0 && p1 == 0.0) {
        *lo = (float)a;
        *hi = (float)b;
        return 1;
    }
    const double U = 2.0 + 0x1p-16;
    const double M = fmax(fabs(a), fabs(b)) + U * (fabs(p0) + fabs(p1));
    const double l = a + U * (fmin(0.0, p0) + fmin(0.0, p1)) - M * 0x1p-20;
    const double h = b + U * (fmax(0.0, p0) + fmax(0.0, p1)) + M * 0x1p-20;
    *lo = (float)l;
    *hi = (float)h;
    if ((double)*lo > l) *lo = nextafterf(*lo, -INFINITY);
    if ((double)*hi < h) *hi = nextafterf(*hi, INFINITY);
    return *lo > -INFINITY && *hi < INFINITY;
}

/* One leaf's constants and the box its accepted hit points lie within delta of.  wrapped = 0: plain
 * leaves only (the reference tree); 1: Transformation / Animation leaves too, with their true world
 * boxes (trees built over those).  Volumes: never.  0 if not cullable; *never = 1 if it can never
 * report a hit. */
static int rtw_cull_leaf(const rtw_world* w, const rtw_leaf* L, int wrapped, float* k, float* m, float lo[3],
                         float hi[3], int* never) {
    *never = 0;
    if (L->flags & RTW_LEAF_VOLUME) return 0;
    const int xf = (L->flags & (RTW_LEAF_TRANSFORM | RTW_LEAF_ANIMATION)) != 0;
    if (xf && !wrapped) return 0;
    if (L->flags & ~(RTW_LEAF_TRANSFORM | RTW_LEAF_ANIMATION)) return 0;
    float llo[3], lhi[3];
    int good = 0;
    const int32_t gi = L->geom_index;
    if (L->geom_kind == RTW_GEOM_SPHERE && gi >= 0 && gi < w->sphere_count) {
        good = rtw_cull_sphere(w->spheres[gi].center, w->spheres[gi].radius, k, m, llo, lhi);
    } else if (L->geom_kind == RTW_GEOM_TRIANGLE && gi >= 0 && gi < w->triangle_count) {
        good = rtw_cull_triangle(w->triangles[gi].positions, k, m, llo, lhi, never);
    } else if (L->geom_kind == RTW_GEOM_RECT && gi >= 0 && gi < w->rect_count) {
        good = rtw_cull_rect(&w->rects[gi], k, m, llo, lhi);
    } else if (L->geom_kind == RTW_GEOM_BOX && gi >= 0 && gi < w->box_count) {
        good = rtw_cull_box(&w->boxes[gi], k, m, llo, lhi);
    }
    if (!good || *never) return good;
    if (!xf) {
        for (int i = 0; i < 3; ++i) { lo[i] = llo[i]; hi[i] = lhi[i]; }
        return 1;
    }
    /* Animation offsets sweep over every ray time, the rolling shutter's included */
    float t0, t1;
    if (!rtw_ray_time_range(&w->camera, &t0, &t1)) return 0;
    if (!rtw_wrap_box(L, t0, t1, llo, lhi, lo, hi)) return 0;
    const float T = rtw_maxr(__builtin_fabsf(t0), __builtin_fabsf(t1));
    float A = 0.0f, off = 0.0f, vel = 0.0f;
    for (int i = 0; i < 3; ++i) {
        A = rtw_maxr(A, rtw_maxr(__builtin_fabsf(lo[i]), __builtin_fabsf(hi[i])));
        if (L->flags & RTW_LEAF_TRANSFORM) off = rtw_maxr(off, __builtin_fabsf(L->offset[i]));
        if (L->flags & RTW_LEAF_ANIMATION) vel = rtw_maxr(vel, __builtin_fabsf(L->velocity[i]));
    }
    const double aw = (double)A > (double)off + (double)vel * T ? (double)A : (double)off + (double)vel * T;
    const double mm = (double)*m + 16.0 * (double)RTW_CULL_U * aw;
    *m = (float)(mm * (1.0 + 0x1p-20));
    return *m < INFINITY;
}

static void rtw_cull_visit(const rtw_world* w, int32_t n, int depth, float* km, rtw_cull_acc* acc, int wrapped) {
    const float inf = rtw_u2f(0x7F800000u);
    if (depth > 64) { acc->ok = 0; return; }
    if (n < 0) {
        const int32_t li = -1 - n;
        if (li >= w->leaf_count) { acc->ok = 0; return; }
        float k = 0.0f, m = 0.0f, lo[3], hi[3];
        int never = 0;
        const int good = rtw_cull_leaf(w, &w->leaves[li], wrapped, &k, &m, lo, hi, &never);
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
    rtw_cull_visit(w, nd->left, depth + 1, km, &sub, wrapped);
    rtw_cull_visit(w, nd->right, depth + 1, km, &sub, wrapped);
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

/* km: 2 * node_count floats.  disable != 0: every node gets k = +inf (reference traversal).
 * wrapped: see rtw_cull_leaf (0 for the reference tree). */
static inline void rtw_cull_prepare_ex(const rtw_world* w, float* km, int disable, int wrapped) {
    const float inf = rtw_u2f(0x7F800000u);
    for (int32_t n = 0; n < w->node_count; ++n) {
        km[2 * (size_t)n] = inf;
        km[2 * (size_t)n + 1] = inf;
    }
    if (disable || w->root < 0) return;
    rtw_cull_acc top;
    rtw_cull_acc_init(&top);
    rtw_cull_visit(w, w->root, 0, km, &top, wrapped);
}
static inline void rtw_cull_prepare(const rtw_world* w, float* km, int disable) {
    rtw_cull_prepare_ex(w, km, disable, 0);
}

#endif /* RTW_CULL_H */
