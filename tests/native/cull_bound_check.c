/* Stress test of the proximity cull's error bound (include/rtw_cull.h, rtw_scalar.h rtw_cull_*,
 * DESIGN.md "Proximity cull").  For random spheres, triangles, rects and box primitives, plain and
 * wrapped in a Y rotation + translation and / or a motion (Transformation / Animation,
 * hittable.rs:234-244) -- grazing/silhouette rays, slivers, near-parallel rays, origins on and far
 * from the surface, scales 1e-2..1e3 -- run the reference's f32 primitive test
 * (sphere_geometry.rs:21-59, triangle_geometry.rs:13-45, rect_geometry.rs:33-59, aabb.rs:80-167)
 * on the ray the device gives the leaf, with t_range [0.001, te).  Every accepted hit must pass the
 * cull predicate on the leaf's own cull box (rtw_cull_leaf: the tightest node that can contain it).
 * Also reports the largest ratio
 *   (distance of the exact point o + t d outside the box) / delta
 * which the bound requires to stay < 1.  Exit status 1 on any violation.
 * Built with -ffp-contract=off like the kernel and the oracle. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/rtw_cull.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

static uint64_t s = 0x243F6A8885A308D3ull;
static inline uint64_t nxt(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline double U(void) { return (double)(nxt() >> 11) * 0x1p-53; }
static inline double R(double a, double b) { return a + (b - a) * U(); }
static inline double LR(double a, double b) { return exp(R(log(a), log(b))); }

typedef struct { float e[3]; } V;
static V sub(V a, V b) { V r = {{a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]}}; return r; }
static V add(V a, V b) { V r = {{a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]}}; return r; }
static V mul(V a, float k) { V r = {{a.e[0] * k, a.e[1] * k, a.e[2] * k}}; return r; }
static float dot(V a, V b) { return (a.e[0] * b.e[0] + a.e[1] * b.e[1]) + a.e[2] * b.e[2]; }
static V cross(V a, V b) {
    V r = {{a.e[1] * b.e[2] - a.e[2] * b.e[1], a.e[2] * b.e[0] - a.e[0] * b.e[2], a.e[0] * b.e[1] - a.e[1] * b.e[0]}};
    return r;
}
static V unit(V a) { return mul(a, 1.0f / sqrtf(dot(a, a))); } /* vec3.rs unit(): v * (1/len) */

static int sphere_hit(V c, float r, V o, V d, float ts, float te, float* t) {
    const V oc = sub(o, c);
    const float hb = dot(oc, d);
    const float cc = dot(oc, oc) - r * r;
    const float disc = hb * hb - cc;
    if (disc < 0.0f) return 0;
    const float sq = sqrtf(disc);
    const float rs = -hb - sq;
    if (ts <= rs && rs < te) { *t = rs; return 1; }
    const float rl = -hb + sq;
    if (ts <= rl && rl < te) { *t = rl; return 1; }
    return 0;
}

static int tri_hit(const V* p, V o, V d, float ts, float te, float* t) {
    const V d1 = sub(p[1], p[0]), d2 = sub(p[2], p[0]);
    const V n = unit(cross(d1, d2));
    const float den = dot(d, n);
    if (!(fabsf(den) > 0.0001f)) return 0;
    const float tt = dot(sub(p[0], o), n) / den;
    if (!(ts <= tt && tt < te)) return 0;
    const V q = sub(add(o, mul(d, tt)), p[0]);
    V vt = cross(n, d2);
    const float w1 = dot(q, vt) / dot(d1, vt);
    if (!(w1 > 0.0f && w1 < 1.0f)) return 0;
    vt = cross(n, d1);
    const float w2 = dot(q, vt) / dot(d2, vt);
    const float w0 = 1.0f - w1 - w2;
    if (!(w2 > 0.0f && w0 > 0.0f)) return 0;
    *t = tt;
    return 1;
}

/* the cull predicate exactly as the oracle / kernel evaluate it (node box = lo, hi) */
static int cull_pass(const float lo[3], const float hi[3], float k, float m, V o, V d, float ts, float te) {
    float ab[6], t0[3], t1[3];
    for (int i = 0; i < 3; ++i) {
        const float a = lo[i] - o.e[i], b = hi[i] - o.e[i];
        ab[2 * i] = a;
        ab[2 * i + 1] = b;
        const float qa = a / d.e[i], qb = b / d.e[i];
        t0[i] = (qa < qb) ? qa : qb;
        t1[i] = (qa < qb) ? qb : qa;
    }
    const float delta = rtw_cull_delta(k, m, ab[0], ab[1], ab[2], ab[3], ab[4], ab[5]);
    float l = ts, h = te;
    for (int i = 0; i < 3; ++i) rtw_cull_axis(t0[i], t1[i], delta * fabsf(1.0f / d.e[i]), &l, &h);
    return l <= h;
}

static double outside(const float lo[3], const float hi[3], V o, V d, float t) {
    double m = 0.0;
    for (int i = 0; i < 3; ++i) {
        const double x = (double)o.e[i] + (double)t * (double)d.e[i];
        const double e = fmax((double)lo[i] - x, x - (double)hi[i]);
        if (e > m) m = e;
    }
    return m;
}
static double delta_of(const float lo[3], const float hi[3], float k, float m, V o) {
    double D = 0.0, Dq = 0.0;
    for (int i = 0; i < 3; ++i) {
        const double mi = fmax(fabs((double)lo[i] - o.e[i]), fabs((double)hi[i] - o.e[i]));
        D += mi;
        Dq += mi * mi;
    }
    return (double)k * Dq + 64.0 * 0x1p-24 * D + (double)m;
}

static V rnd_dir(void) {
    V d;
    do {
        for (int i = 0; i < 3; ++i) d.e[i] = (float)R(-1, 1);
    } while (dot(d, d) > 1.0f || dot(d, d) < 1e-3f);
    return unit(d);
}

static int rect_hit(const rtw_rect* g, V o, V d, float ts, float te, float* t) {
    int p0, p1, n;
    rtw_rect_axes(g->plane, &p0, &p1, &n);
    const float tt = (g->dist - o.e[n]) / d.e[n];
    if (!(ts <= tt && tt < te)) return 0;
    const V pos = add(o, mul(d, tt));
    if (!(pos.e[p0] >= g->r0[0] && pos.e[p0] <= g->r0[1] && pos.e[p1] >= g->r1[0] && pos.e[p1] <= g->r1[1])) return 0;
    *t = tt;
    return 1;
}

static int box_hit(const rtw_box* b, V o, V d, float ts, float te, float* t) { /* aabb.rs:80-167 */
    float near = -INFINITY, far = INFINITY;
    for (int a = 0; a < 3; ++a) {
        const float t1 = (b->min[a] - o.e[a]) / d.e[a], t2 = (b->max[a] - o.e[a]) / d.e[a];
        const float tmin = rtw_minr(t1, t2), tmax = rtw_maxr(t1, t2);
        if (tmin > near) near = tmin;
        if (tmax < far) far = tmax;
        if (near > far || far < 0.0f) return 0;
    }
    if (ts <= near && near < te) { *t = near; return 1; }
    if (ts <= far && far < te) { *t = far; return 1; }
    return 0;
}

/* the device's leaf_local_ray: Animation (outermost) then Transformation, xf_reverse each */
static void local_ray(const rtw_leaf* L, float time, V o, V d, V* lo, V* ld) {
    if (L->flags & RTW_LEAF_ANIMATION) {
        const V vt = mul((V){{L->velocity[0], L->velocity[1], L->velocity[2]}}, time);
        const V off = {{0.0f + vt.e[0], 0.0f + vt.e[1], 0.0f + vt.e[2]}};
        o = sub(o, off);  /* rot_up(1, -0, .) is exact */
    }
    if (L->flags & RTW_LEAF_TRANSFORM) {
        const float c = L->y_cos, sn = -L->y_sin;
        const V q = sub(o, (V){{L->offset[0], L->offset[1], L->offset[2]}});
        o = (V){{c * q.e[0] + sn * q.e[2], q.e[1], -sn * q.e[0] + c * q.e[2]}};
        d = (V){{c * d.e[0] + sn * d.e[2], d.e[1], -sn * d.e[0] + c * d.e[2]}};
    }
    *lo = o;
    *ld = d;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 2000000;
    long acc_s = 0, acc_t = 0, bad = 0;
    double worst_s = 0.0, worst_t = 0.0;
    for (long it = 0; it < n; ++it) {  /* spheres */
        const double S = LR(1e-2, 1e3);
        V c;
        for (int i = 0; i < 3; ++i) c.e[i] = (float)(R(-1, 1) * S * LR(1e-3, 1e3));
        const float r = (float)(S * LR(1e-3, 1));
        const double dist = (nxt() & 1) ? r * LR(1, 1e4) : r * (1.0 + R(-1, 1) * LR(1e-7, 1e-1));
        const V o = add(c, mul(rnd_dir(), (float)dist));
        const float eps = (float)(R(-1, 1) * LR(1e-9, 1e-2));
        const V d = unit(sub(add(c, mul(rnd_dir(), r * (1.0f + eps))), o));
        const float te = (nxt() & 3) ? INFINITY : (float)(dist * LR(0.5, 2.0));
        float t, k, m, lo[3], hi[3];
        if (!sphere_hit(c, r, o, d, 0.001f, te, &t)) continue;
        if (!rtw_cull_sphere(c.e, r, &k, &m, lo, hi)) continue;
        ++acc_s;
        if (!cull_pass(lo, hi, k, m, o, d, 0.001f, te)) ++bad;
        const double q = outside(lo, hi, o, d, t) / delta_of(lo, hi, k, m, o);
        if (q > worst_s) worst_s = q;
    }
    for (long it = 0; it < n; ++it) {  /* triangles */
        const double S = LR(1e-2, 1e3);
        V p[3];
        double base[3];
        for (int i = 0; i < 3; ++i) base[i] = R(-1, 1) * S * LR(1e-3, 1e3);
        for (int j = 0; j < 3; ++j)
            for (int i = 0; i < 3; ++i) p[j].e[i] = (float)(base[i] + R(-1, 1) * S);
        if (nxt() & 1) {  /* sliver: p2 near the line p0 p1 */
            const double a = R(0, 1), h = LR(1e-5, 1);
            const V off = rnd_dir();
            for (int i = 0; i < 3; ++i) p[2].e[i] = (float)(p[0].e[i] + a * (p[1].e[i] - p[0].e[i]) + h * S * off.e[i]);
        }
        double e1[3], e2[3], nn[3];
        for (int i = 0; i < 3; ++i) { e1[i] = (double)p[1].e[i] - p[0].e[i]; e2[i] = (double)p[2].e[i] - p[0].e[i]; }
        nn[0] = e1[1] * e2[2] - e1[2] * e2[1];
        nn[1] = e1[2] * e2[0] - e1[0] * e2[2];
        nn[2] = e1[0] * e2[1] - e1[1] * e2[0];
        const double nl = sqrt(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
        if (!(nl > 0.0)) continue;
        double w1 = R(0, 1), w2 = R(0, 1 - w1);
        const int mode = (int)(nxt() % 3);
        if (mode == 0) w2 = 0.0;
        else if (mode == 1) { w1 = 0.0; w2 = R(0, 1); }
        else w2 = 1.0 - w1;
        const double diam = sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]) + sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
        double tgt[3];
        for (int i = 0; i < 3; ++i) tgt[i] = p[0].e[i] + w1 * e1[i] + w2 * e2[i] + R(-1, 1) * LR(1e-9, 1e-3) * diam;
        V dd = rnd_dir();
        if (nxt() & 1) {  /* nearly in-plane direction */
            const double dn = (dd.e[0] * nn[0] + dd.e[1] * nn[1] + dd.e[2] * nn[2]) / nl;
            const double keep = LR(1e-5, 1e-1);
            double v[3], l = 0.0;
            for (int i = 0; i < 3; ++i) { v[i] = dd.e[i] - dn * nn[i] / nl + keep * nn[i] / nl; l += v[i] * v[i]; }
            for (int i = 0; i < 3; ++i) dd.e[i] = (float)(v[i] / sqrt(l));
        }
        const double dist = diam * LR(1e-2, 1e4);
        V o, tv;
        for (int i = 0; i < 3; ++i) { o.e[i] = (float)(tgt[i] + dist * dd.e[i]); tv.e[i] = (float)tgt[i]; }
        const V d = unit(sub(tv, o));
        const float te = (nxt() & 3) ? INFINITY : (float)(dist * LR(0.5, 2.0));
        float t, k, m, lo[3], hi[3];
        int never = 0;
        if (!tri_hit(p, o, d, 0.001f, te, &t)) continue;
        float pp[3][3];
        for (int j = 0; j < 3; ++j)
            for (int i = 0; i < 3; ++i) pp[j][i] = p[j].e[i];
        if (!rtw_cull_triangle(pp, &k, &m, lo, hi, &never)) continue;
        if (never) { ++bad; continue; } /* a "never" triangle reported a hit */
        ++acc_t;
        if (!cull_pass(lo, hi, k, m, o, d, 0.001f, te)) ++bad;
        const double q = outside(lo, hi, o, d, t) / delta_of(lo, hi, k, m, o);
        if (q > worst_t) worst_t = q;
    }
    /* rects, boxes and spheres, plain or wrapped (rtw_cull_leaf with wrapped = 1) */
    long acc_w[3] = {0, 0, 0};
    double worst_w[3] = {0.0, 0.0, 0.0};
    const char* wname[3] = {"rect", "box", "wrapped"};
    for (long it = 0; it < n; ++it) {
        const double S = LR(1e-2, 1e3);
        double base[3];
        for (int i = 0; i < 3; ++i) base[i] = R(-1, 1) * S * LR(1e-3, 1e3);
        rtw_sphere sp;
        rtw_rect rc;
        rtw_box bx;
        rtw_leaf L = {0};
        rtw_world w = {0};
        const int kind = (int)(nxt() % 3);  /* 0 rect, 1 box, 2 sphere */
        double tgt[3];                      /* a local point on the primitive's surface */
        if (kind == 0) {
            rc.plane = (int32_t)(nxt() % 3);
            int p0, p1, nn;
            rtw_rect_axes(rc.plane, &p0, &p1, &nn);
            rc.dist = (float)base[nn];
            const double a0 = base[p0], a1 = base[p0] + S * LR(1e-3, 1), b0 = base[p1], b1 = base[p1] + S * LR(1e-3, 1);
            rc.r0[0] = (float)a0; rc.r0[1] = (float)a1; rc.r1[0] = (float)b0; rc.r1[1] = (float)b1;
            tgt[nn] = rc.dist;
            const int edge = (int)(nxt() % 3);  /* interior, near the p0 edges, near the p1 edges */
            tgt[p0] = edge == 1 ? ((nxt() & 1) ? a0 : a1) + R(-1, 1) * LR(1e-9, 1e-4) * S : R(a0, a1);
            tgt[p1] = edge == 2 ? ((nxt() & 1) ? b0 : b1) + R(-1, 1) * LR(1e-9, 1e-4) * S : R(b0, b1);
            L.geom_kind = RTW_GEOM_RECT;
            w.rects = &rc;
            w.rect_count = 1;
        } else if (kind == 1) {
            for (int i = 0; i < 3; ++i) {
                bx.min[i] = (float)base[i];
                bx.max[i] = (float)(base[i] + S * LR(1e-3, 1));
            }
            const int face = (int)(nxt() % 3);
            for (int i = 0; i < 3; ++i) tgt[i] = R(bx.min[i], bx.max[i]);
            tgt[face] = (nxt() & 1) ? bx.min[face] : bx.max[face];
            if (nxt() & 1) {  /* near an edge */
                const int e2 = (face + 1 + (int)(nxt() & 1)) % 3;
                tgt[e2] = ((nxt() & 1) ? bx.min[e2] : bx.max[e2]) + R(-1, 1) * LR(1e-9, 1e-4) * S;
            }
            L.geom_kind = RTW_GEOM_BOX;
            w.boxes = &bx;
            w.box_count = 1;
        } else {
            for (int i = 0; i < 3; ++i) sp.center[i] = (float)base[i];
            sp.radius = (float)(S * LR(1e-3, 1));
            const V u = rnd_dir();
            for (int i = 0; i < 3; ++i) tgt[i] = sp.center[i] + sp.radius * (1.0 + R(-1, 1) * LR(1e-9, 1e-3)) * u.e[i];
            L.geom_kind = RTW_GEOM_SPHERE;
            w.spheres = &sp;
            w.sphere_count = 1;
        }
        const int wrapped = kind == 2 || (nxt() & 1);
        float time = 0.0f;
        w.camera.time0 = 0.0f;
        w.camera.time1 = (nxt() & 1) ? 0.0f : (float)LR(1e-2, 4.0);
        if (wrapped) {
            const int fl = 1 + (int)(nxt() % 3);  /* transform, animation, both */
            if (fl & 1) {
                L.flags |= RTW_LEAF_TRANSFORM;
                const double ang = R(-M_PI, M_PI);
                L.y_cos = (float)cos(ang);
                L.y_sin = (float)sin(ang);
                for (int i = 0; i < 3; ++i) L.offset[i] = (float)(R(-1, 1) * S * LR(1e-3, 1e3));
            }
            if (fl & 2) {
                L.flags |= RTW_LEAF_ANIMATION;
                for (int i = 0; i < 3; ++i) L.velocity[i] = (float)(R(-1, 1) * S * LR(1e-3, 10));
                time = (float)R(w.camera.time0, w.camera.time1);
            }
        }
        /* the target's world position (exact forward map of the local point) */
        double wt[3] = {tgt[0], tgt[1], tgt[2]};
        if (L.flags & RTW_LEAF_TRANSFORM) {
            const double c = L.y_cos, sn = L.y_sin, det = c * c + sn * sn;
            const double x = wt[0], z = wt[2];
            wt[0] = (c * x + sn * z) / det + L.offset[0];
            wt[1] += L.offset[1];
            wt[2] = (-sn * x + c * z) / det + L.offset[2];
        }
        if (L.flags & RTW_LEAF_ANIMATION)
            for (int i = 0; i < 3; ++i) wt[i] += (double)L.velocity[i] * (double)time;
        V dd = rnd_dir();
        const double dist = S * LR(1e-3, 1e4);
        V o, tv;
        for (int i = 0; i < 3; ++i) { o.e[i] = (float)(wt[i] + dist * dd.e[i]); tv.e[i] = (float)wt[i]; }
        const V d = unit(sub(tv, o));
        const float te = (nxt() & 3) ? INFINITY : (float)(dist * LR(0.5, 2.0));
        V lo_, ld_;
        local_ray(&L, time, o, d, &lo_, &ld_);
        float t;
        const int hit = kind == 0 ? rect_hit(&rc, lo_, ld_, 0.001f, te, &t)
                      : kind == 1 ? box_hit(&bx, lo_, ld_, 0.001f, te, &t)
                                  : sphere_hit((V){{sp.center[0], sp.center[1], sp.center[2]}}, sp.radius, lo_, ld_, 0.001f, te, &t);
        if (!hit) continue;
        float k, m, lo[3], hi[3];
        int never = 0;
        if (!rtw_cull_leaf(&w, &L, 1, &k, &m, lo, hi, &never) || never) continue;
        const int cls = wrapped ? 2 : kind;  /* plain spheres are covered above */
        ++acc_w[cls];
        if (!cull_pass(lo, hi, k, m, o, d, 0.001f, te)) ++bad;
        const double q = outside(lo, hi, o, d, t) / delta_of(lo, hi, k, m, o);
        if (q > worst_w[cls]) worst_w[cls] = q;
    }
    printf("sphere hits %ld (max outside/delta %.4f), triangle hits %ld (max outside/delta %.4f)", acc_s, worst_s,
           acc_t, worst_t);
    for (int c = 0; c < 3; ++c) printf(", %s hits %ld (max outside/delta %.4f)", wname[c], acc_w[c], worst_w[c]);
    printf(", violations %ld\n", bad);
    return bad == 0 && worst_s < 1.0 && worst_t < 1.0 && worst_w[0] < 1.0 && worst_w[1] < 1.0 && worst_w[2] < 1.0 ? 0 : 1;
}
