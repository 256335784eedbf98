"""Generates the golden fixtures in tests/golden/ (run here, in the build container; the
committed outputs are data only -- inputs and expected outputs).

The reference (Rust) cannot be built or run in this image and ships no tests or fixtures, so
these vectors pin our restatements against each other and against regressions:

  rng.json           the published rand_xoshiro 0.6.0 Xoroshiro128PlusPlus vector (seed words 1,
                     2), the "ctr" per-(pixel, sample) stream states (include/rtw_scalar.h) and
                     rand 0.8.5 draws, from the pure-Python restatement (oracle/pyref.py)
  scene1.npz         demo_worlds.rs:395-463 final_scene1 sphere table (pyref) and the BVH
                     hittable.rs:360-427 builds over it (pyref.bvh_build)
  hits.npz           primitive hit known-answer tests: sphere_geometry.rs:21-59,
                     rect_geometry.rs:33-59, aabb.rs:80-167, triangle_geometry.rs:13-45 restated
                     below in numpy f32 one operation at a time (no FMA), on random rays aimed at
                     one primitive each
  images.npz         tiny frames rendered by the C oracle in ctr mode (regression pin of the whole
                     loop; the GPU must reproduce them bit for bit)

python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import pyoracle as O  # noqa: E402
from oracle import pyref  # noqa: E402

import raytracinginaweekend_amd as R  # noqa: E402

f32 = np.float32
M64 = (1 << 64) - 1

IMAGES = [  # name, width, height, spp, max_depth, seed
    ("final_scene1", 32, 18, 4, 50, 3),
    ("suzanne", 32, 18, 2, 50, 3),
    ("cornell_box", 24, 24, 4, 50, 3),
    ("cornell_cube", 24, 24, 4, 50, 3),
    ("final_scene2", 24, 24, 2, 50, 3),
    ("earth_mapped", 32, 18, 2, 50, 3),
    ("cornell_box_smoke", 24, 24, 2, 50, 3),
]


# ------------------------------------------------------------------------------------------------
def mix64(z: int) -> int:
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def sample_stream(seed: int, pixel: int, sample: int) -> tuple[int, int]:
    key = mix64((seed ^ 0x5EED5EED5EED5EED) & M64)
    x = mix64(((pixel << 32) | sample) ^ key)
    s0 = x
    s1 = ((x ^ (x >> 32)) * 0xD6E8FEB86659FD93) & M64
    return (s0 or 1) if (s0 | s1) == 0 else s0, s1


def rng_fixture() -> dict:
    r = pyref.Xoro(1, 2)
    kat = [r.next_u64() for _ in range(9)]
    streams = []
    for seed, pixel, sample in [(0x5EED, 0, 0), (0x5EED, 12345, 511), (7, 2073599, 0), (2**63 + 5, 99, 3)]:
        s0, s1 = sample_stream(seed, pixel, sample)
        x = pyref.Xoro(s0, s1)
        draws = {
            "u64": [x.next_u64() for _ in range(4)],
            "f32": [float(x.gen_f32()) for _ in range(4)],
            "range_0_1": [float(x.gen_range_f32(0.0, 1.0)) for _ in range(2)],
            "unit_sphere": [float(v) for v in x.unit_sphere()],
            "unit_disc": [float(v) for v in x.unit_disc()],
            "unit_ball": [float(v) for v in x.unit_ball()],
        }
        streams.append({"seed": seed, "pixel": pixel, "sample": sample, "s0": s0, "s1": s1, "draws": draws})
    return {"xoroshiro128pp_seed_1_2": kat, "ctr_streams": streams}


# ------------------------------------------------------------------------------------------------
def scene1_fixture() -> dict:
    sph = pyref.final_scene1_spheres()
    centers = np.array([s[0] for s in sph], np.float32)
    radii = np.array([s[1] for s in sph], np.float32)
    kinds = np.array([{"lambert": 0, "metal": 1, "dielectric": 2}[s[2][0]] for s in sph], np.int32)
    albedo = np.array([s[2][1] if s[2][0] != "dielectric" else (0, 0, 0) for s in sph], np.float32)
    fuzz = np.array([s[2][2] if s[2][0] == "metal" else 0 for s in sph], np.float32)
    boxes = [pyref.sphere_box(c, r) for c, r in zip(centers, radii)]
    root, nodes = pyref.bvh_build(boxes)
    return dict(centers=centers, radii=radii, kinds=kinds, albedo=albedo, fuzz=fuzz, bvh_root=np.int32(root),
                bvh_min=np.array([n[0] for n in nodes], np.float32), bvh_max=np.array([n[1] for n in nodes], np.float32),
                bvh_axis=np.array([n[2] for n in nodes], np.int32),
                bvh_children=np.array([[n[3], n[4]] for n in nodes], np.int32))


# ------------------------------------------------------------------------------------------------
# primitive restatements in numpy f32
def v(*a):
    return [f32(x) for x in a]


def vsub(a, b):
    return [a[0] - b[0], a[1] - b[1], a[2] - b[2]]


def vadd(a, b):
    return [a[0] + b[0], a[1] + b[1], a[2] + b[2]]


def vmul(a, s):
    return [a[0] * s, a[1] * s, a[2] * s]


def dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def cross(a, b):
    return [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]


def unit(a):  # vec3.rs:205-210: v * (1 / len)
    return vmul(a, f32(1.0) / np.sqrt(dot(a, a)))


def contains(t, ts, te):
    return ts <= t < te


def front(sn, d):  # hittable.rs:33-54
    ff = dot(sn, d) < f32(0.0)
    return (sn if ff else [-sn[0], -sn[1], -sn[2]]), ff


def hit_sphere(c, r, o, d, ts, te):
    oc = vsub(o, c)
    hb = dot(oc, d)
    cc = dot(oc, oc) - r * r
    disc = hb * hb - cc
    if disc < f32(0.0):
        return None
    sq = np.sqrt(disc)
    t = -hb - sq
    if not contains(t, ts, te):
        t = -hb + sq
        if not contains(t, ts, te):
            return None
    pos = vadd(o, vmul(d, t))
    sn = [x / r for x in vsub(pos, c)]
    return t, pos, sn


def hit_rect(plane, dist, r0, r1, o, d, ts, te):
    p0, p1, n = {0: (0, 1, 2), 1: (0, 2, 1), 2: (1, 2, 0)}[plane]  # XY, XZ, YZ
    t = (dist - o[n]) / d[n]
    if not contains(t, ts, te):
        return None
    pos = vadd(o, vmul(d, t))
    if not (pos[p0] >= r0[0] and pos[p0] <= r0[1] and pos[p1] >= r1[0] and pos[p1] <= r1[1]):
        return None
    sn = [f32(0.0)] * 3
    sn[n] = f32(-1.0)
    return t, pos, sn


def rmin(a, b):  # Rust f32::min: the non-NaN operand
    return b if np.isnan(a) else (a if np.isnan(b) else (a if a < b else b))


def rmax(a, b):
    return b if np.isnan(a) else (a if np.isnan(b) else (a if a > b else b))


def hit_box(mn, mx, o, d, ts, te):
    lo, hi = vsub(mn, o), vsub(mx, o)
    near, far, npl, fpl = f32(-np.inf), f32(np.inf), 0, 0
    for a in range(3):
        with np.errstate(divide="ignore", invalid="ignore"):
            t1, t2 = lo[a] / d[a], hi[a] / d[a]
        tmin, tmax = rmin(t1, t2), rmax(t1, t2)
        if tmin > near:
            near, npl = tmin, a
        if tmax < far:
            far, fpl = tmax, a
        if near > far or far < f32(0.0):
            return None
    if contains(near, ts, te):
        t, plane = near, npl
    elif contains(far, ts, te):
        t, plane = far, fpl
    else:
        return None
    pos = vadd(o, vmul(d, t))
    center = (mx[plane] + mn[plane]) * f32(0.5)
    sn = [f32(0.0)] * 3
    x = pos[plane] - center
    sn[plane] = f32(1.0) if x > 0 else (f32(-1.0) if x < 0 else (f32(np.copysign(1.0, x)) if x == 0 else x))
    return t, pos, sn


def hit_tri(p, nrm, o, d, ts, te):
    d1, d2 = vsub(p[1], p[0]), vsub(p[2], p[0])
    n = unit(cross(d1, d2))
    den = dot(d, n)
    if not (abs(den) > f32(0.0001)):
        return None
    t = dot(vsub(p[0], o), n) / den
    if not contains(t, ts, te):
        return None
    pos = vadd(o, vmul(d, t))
    q = vsub(pos, p[0])
    vt = cross(n, d2)
    w1 = dot(q, vt) / dot(d1, vt)
    if not (w1 > f32(0.0) and w1 < f32(1.0)):
        return None
    vt = cross(n, d1)
    w2 = dot(q, vt) / dot(d2, vt)
    w0 = f32(1.0) - w1 - w2
    if not (w2 > f32(0.0) and w0 > f32(0.0)):
        return None
    sn = vadd(vadd(vmul(nrm[0], w0), vmul(nrm[1], w1)), vmul(nrm[2], w2))  # math.rs:9-16
    return t, pos, sn


def one_leaf_world(kind: str, rng):
    wb = R.WorldBuilder()
    m = wb.material_lambert_solid((0.5, 0.5, 0.5))
    if kind == "sphere":
        node = wb.new_obj_sphere(float(rng.uniform(0.3, 2.0)), m).translate(tuple(rng.uniform(-2, 2, 3)))
    elif kind == "rect":
        node = [wb.new_obj_rect_xy, wb.new_obj_rect_xz, wb.new_obj_rect_yz][rng.integers(3)](
            tuple(rng.uniform(-2, 2, 3)), float(rng.uniform(0.5, 3)), float(rng.uniform(0.5, 3)), m)
    elif kind == "box":
        node = wb.new_obj_box(*[float(x) for x in rng.uniform(0.5, 3, 3)], m).translate(tuple(rng.uniform(-2, 2, 3)))
    else:
        tri = np.zeros((1, 24), np.float32)
        tri[0, :9] = rng.uniform(-2, 2, 9)
        tri[0, 9:18] = rng.uniform(-1, 1, 9)
        tri[0, 18:] = rng.uniform(0, 1, 6)
        node = wb.new_mesh(tri, m)
    cam = R.Camera.build().vertical_fov(40.0, 1.0).position((0, 0, 10)).look_at((0, 0, 0), (0, 1, 0)).build()
    return node.build().finish(wb, R.BackgroundColor.sky(), cam)


def aim(rng, target):
    o = rng.uniform(-8, 8, 3).astype(np.float32)
    tgt = np.asarray(target, np.float64) + rng.normal(0, 0.6, 3)
    return [f32(x) for x in o], unit([f32(x) for x in (tgt - o).astype(np.float32)])


def hits_fixture() -> dict:
    rng = np.random.default_rng(20261015)
    out = {k: [] for k in ("kind", "prim", "origin", "dir", "hit", "t", "pos", "normal", "front")}
    prims = []
    for kind in ("sphere", "rect", "box", "triangle"):
        for w_i in range(6):
            world = one_leaf_world(kind, rng)
            raw = world.raw
            if kind == "sphere":
                s = raw.spheres[0]
                c, r = v(*s.center), f32(s.radius)
                prim = list(c) + [r]
                target = c
                fn = lambda o, d: hit_sphere(c, r, o, d, f32(0.001), f32(np.inf))  # noqa: E731
            elif kind == "rect":
                g = raw.rects[0]
                prim = [g.plane, g.dist, g.r0[0], g.r0[1], g.r1[0], g.r1[1]]
                p0, p1, n = {0: (0, 1, 2), 1: (0, 2, 1), 2: (1, 2, 0)}[g.plane]
                target = [0.0] * 3
                target[p0], target[p1], target[n] = (g.r0[0] + g.r0[1]) / 2, (g.r1[0] + g.r1[1]) / 2, g.dist
                fn = lambda o, d, g=g: hit_rect(g.plane, f32(g.dist), v(*g.r0), v(*g.r1), o, d, f32(0.001),  # noqa: E731
                                                f32(np.inf))
            elif kind == "box":
                b = raw.boxes[0]
                mn, mx = v(*b.min), v(*b.max)
                prim = list(mn) + list(mx)
                target = [(a + b_) / 2 for a, b_ in zip(mn, mx)]
                fn = lambda o, d: hit_box(mn, mx, o, d, f32(0.001), f32(np.inf))  # noqa: E731
            else:
                t_ = raw.triangles[0]
                p = [v(*t_.positions[i]) for i in range(3)]
                nr = [v(*t_.normals[i]) for i in range(3)]
                prim = [x for q in p for x in q] + [x for q in nr for x in q] + [x for i in range(3) for x in t_.uvs[i]]
                target = [sum(q[i] for q in p) / 3 for i in range(3)]
                fn = lambda o, d: hit_tri(p, nr, o, d, f32(0.001), f32(np.inf))  # noqa: E731
            prims.append((kind, prim, world))
            for _ in range(60):
                o, d = aim(rng, target)
                res = fn(o, d)
                out["kind"].append(["sphere", "rect", "box", "triangle"].index(kind))
                out["prim"].append(len(prims) - 1)
                out["origin"].append(o)
                out["dir"].append(d)
                if res is None:
                    out["hit"].append(0)
                    out["t"].append(f32(0))
                    out["pos"].append([f32(0)] * 3)
                    out["normal"].append([f32(0)] * 3)
                    out["front"].append(0)
                else:
                    t, pos, sn = res
                    n, ff = front(sn, d)
                    out["hit"].append(1)
                    out["t"].append(t)
                    out["pos"].append(pos)
                    out["normal"].append(n)
                    out["front"].append(int(ff))
    fx = {k: np.array(vv, np.float32 if k in ("t", "pos", "normal", "origin", "dir") else np.int32)
          for k, vv in out.items()}
    fx["prim_params"] = np.array([p + [0.0] * (24 - len(p)) for _, p, _ in prims], np.float32)
    fx["prim_kind"] = np.array([["sphere", "rect", "box", "triangle"].index(k) for k, _, _ in prims], np.int32)
    return fx, prims


def images_fixture() -> dict:
    out = {}
    for name, w, h, spp, depth, seed in IMAGES:
        world = R.demo_world(name)
        p = R.render_params(R.Size2i(w, h), spp, depth, seed=seed)
        out[name] = O.render(world, p, O.RNG_CTR, 8)
    return out


def main():
    with open(os.path.join(HERE, "rng.json"), "w") as f:
        json.dump(rng_fixture(), f, indent=1)
    np.savez_compressed(os.path.join(HERE, "scene1.npz"), **scene1_fixture())
    fx, _ = hits_fixture()
    np.savez_compressed(os.path.join(HERE, "hits.npz"), **fx)
    np.savez_compressed(os.path.join(HERE, "images.npz"), **images_fixture())
    print("hits:", int(fx["hit"].sum()), "of", len(fx["hit"]))


if __name__ == "__main__":
    main()
