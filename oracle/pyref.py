"""TEST INFRASTRUCTURE: pure-Python restatement of the reference's host-side algorithms.

Independent of librtw.so's C++ builder, used by tests/ to check it:
  * Xoroshiro128PlusPlus + rand 0.8.5 sampling (rand_xoshiro 0.6.0 / rand 0.8.5; not vendored
    under /root/reference -- restated from the published crate algorithms)
  * obj_loader.rs:214-270 (the fan-triangulation quirk)
  * hittable.rs:360-427 BoundingVolumeHierarchy::new/_new, aabb.rs bounding boxes
  * demo_worlds.rs:395-463 create_world_final_scene1 (the random sphere table)
f32 arithmetic is done with numpy.float32 scalars, one operation at a time.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32
M64 = (1 << 64) - 1


# ------------------------------------------------------------------------------------------------
# RNG
# ------------------------------------------------------------------------------------------------
def _rotl(x: int, k: int) -> int:
    return ((x << k) | (x >> (64 - k))) & M64


class Xoro:
    """Xoroshiro128PlusPlus (rand_xoshiro 0.6.0)."""

    def __init__(self, s0: int, s1: int):
        self.s0, self.s1 = s0 & M64, s1 & M64

    @classmethod
    def from_seed(cls, seed: bytes) -> "Xoro":
        return cls(int.from_bytes(seed[:8], "little"), int.from_bytes(seed[8:16], "little"))

    def next_u64(self) -> int:
        s0, s1 = self.s0, self.s1
        result = (_rotl((s0 + s1) & M64, 17) + s0) & M64
        s1 ^= s0
        self.s0 = _rotl(s0, 49) ^ s1 ^ ((s1 << 21) & M64)
        self.s1 = _rotl(s1, 28)
        return result

    def next_u32(self) -> int:
        return self.next_u64() & 0xFFFFFFFF

    def gen_f32(self) -> np.float32:  # Standard f32: (u32 >> 8) * 2^-24
        return f32(1.0 / 16777216.0) * f32(self.next_u32() >> 8)

    def _value0_1(self) -> np.float32:
        bits = np.uint32((self.next_u32() >> 9) | 0x3F800000)
        return bits.view(np.float32) - f32(1.0)

    def gen_range_f32(self, low, high) -> np.float32:  # UniformFloat::sample_single
        low, high = f32(low), f32(high)
        scale = high - low
        while True:
            res = self._value0_1() * scale + low
            if res < high:
                return res

    def gen_range_u32(self, n: int) -> int:  # UniformInt::sample_single_inclusive(0, n-1)
        rng = n & 0xFFFFFFFF
        lz = 32 - rng.bit_length()
        zone = ((rng << lz) & 0xFFFFFFFF) - 1
        while True:
            v = self.next_u32()
            m = v * rng
            hi, lo = m >> 32, m & 0xFFFFFFFF
            if lo <= zone:
                return hi

    def uniform_m1_1(self) -> np.float32:
        return self._value0_1() * f32(2.0) + f32(-1.0)

    def unit_sphere(self):
        while True:
            x1, x2 = self.uniform_m1_1(), self.uniform_m1_1()
            s = x1 * x1 + x2 * x2
            if s >= f32(1.0):
                continue
            factor = f32(2.0) * np.sqrt(f32(1.0) - s)
            return [x1 * factor, x2 * factor, f32(1.0) - f32(2.0) * s]

    def unit_ball(self):
        while True:
            x = [self.uniform_m1_1() for _ in range(3)]
            if x[0] * x[0] + x[1] * x[1] + x[2] * x[2] <= f32(1.0):
                return x

    def unit_disc(self):
        while True:
            x1, x2 = self.uniform_m1_1(), self.uniform_m1_1()
            if x1 * x1 + x2 * x2 <= f32(1.0):
                return [x1, x2]


# ------------------------------------------------------------------------------------------------
# OBJ loader (obj_loader.rs)
# ------------------------------------------------------------------------------------------------
def load_obj(text: str) -> np.ndarray:
    """(n, 24) f32: positions(3x3) normals(3x3) uvs(3x2), the fan quirk of :251-264 kept."""
    pos, nor, uv, tris = [], [], [], []
    for line in text.split("\n"):
        line = line.rstrip("\r")
        if line.startswith("vn"):
            nor.append([f32(x) for x in line.split()[1:4]])
        elif line.startswith("vt"):
            uv.append([f32(x) for x in line.split()[1:3]])
        elif line.startswith("v"):
            pos.append([f32(x) for x in line.split()[1:4]])
        elif line.startswith("f"):
            tri = [[f32(0)] * 3, [f32(0)] * 3, [f32(0)] * 3]
            tn = [[f32(0)] * 3, [f32(0)] * 3, [f32(0)] * 3]
            tu = [[f32(0)] * 2, [f32(0)] * 2, [f32(0)] * 2]
            for i, vert in enumerate(line.split()[1:]):
                parts = vert.split("/")
                p = pos[int(parts[0]) - 1]
                t = uv[int(parts[1]) - 1] if len(parts) > 1 and parts[1] else [f32(0), f32(0)]
                n = nor[int(parts[2]) - 1]
                if i < 2:
                    tri[i], tn[i], tu[i] = p, n, t
                else:
                    tri[1], tn[1], tu[1] = tri[2], tn[2], tu[2]
                    tri[2], tn[2], tu[2] = p, n, t
                    tris.append(sum(tri, []) + sum(tn, []) + sum(tu, []))
    return np.array(tris, np.float32).reshape(-1, 24)


# ------------------------------------------------------------------------------------------------
# BVH (hittable.rs:360-427)
# ------------------------------------------------------------------------------------------------
def surrounding(a, b):
    amin, amax = a
    bmin, bmax = b
    return (np.minimum(amin, bmin), np.maximum(amax, bmax))


def bvh_build(boxes):
    """boxes: list of (min[3], max[3]) f32 arrays for leaves 0..n-1.
    Returns (root, nodes) with nodes = [(min, max, axis, left, right)], leaves as -1-i."""
    nodes = []

    def new(items, axis):
        if len(items) == 1:
            return items[0][0], items[0][1]
        items.sort(key=lambda it: it[1][0][axis])  # list.sort is stable, like slice::sort_by
        if len(items) == 2:
            nid = len(nodes)
            bb = surrounding(items[0][1], items[1][1])
            nodes.append((bb[0], bb[1], axis, items[0][0], items[1][0]))
            return nid, bb
        mid = len(items) // 2
        left, right = items[:mid], items[mid:]
        nid = len(nodes)
        nodes.append(None)
        lid, lb = new(left, (axis + len(left)) % 3)
        rid, rb = new(right, (axis + len(right)) % 3)
        items[:mid], items[mid:] = left, right
        bb = surrounding(lb, rb)
        nodes[nid] = (bb[0], bb[1], axis, lid, rid)
        return nid, bb

    items = [(-1 - i, (np.asarray(b[0], np.float32), np.asarray(b[1], np.float32))) for i, b in enumerate(boxes)]
    root, _ = new(items, 0)
    return root, nodes


def sphere_box(center, radius):
    c = np.asarray(center, np.float32)
    r = f32(radius)
    return (c - np.array([r, r, r], np.float32), c + np.array([r, r, r], np.float32))


# ------------------------------------------------------------------------------------------------
# demo_worlds.rs:395-463 final_scene1 sphere table
# ------------------------------------------------------------------------------------------------
def final_scene1_spheres():
    """[(center xyz, radius, material tuple)] in builder order (ground first)."""
    rng = Xoro.from_seed(bytes(range(1, 17)))
    R = f32(1000.0)
    gc = np.array([0.0, -1000.0, 0.0], np.float32)
    out = [((f32(0.0), f32(0.0) - R, f32(0.0)), R, ("lambert", (f32(0.5), f32(0.5), f32(0.5))))]
    for a in range(-11, 12):
        for b in range(-11, 12):
            ox = rng.gen_f32() * f32(0.9)
            oz = rng.gen_f32() * f32(0.9)
            c = np.array([f32(a) + ox, f32(0.2) + f32(0.0), f32(b) + oz], np.float32)
            d = c - np.array([4.0, 0.2, 0.0], np.float32)
            length = np.sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])
            if length > f32(0.9):
                sample = rng.gen_f32()
                if sample < f32(0.8):
                    c1 = [rng.gen_f32() for _ in range(3)]
                    c2 = [rng.gen_f32() for _ in range(3)]
                    mat = ("lambert", tuple(x * y for x, y in zip(c1, c2)))
                elif sample < f32(0.95):
                    col = tuple(rng.gen_f32() for _ in range(3))
                    mat = ("metal", col, rng.gen_range_f32(0.0, 0.5))
                else:
                    mat = ("dielectric", f32(1.5))
                v = c - gc
                ln = np.sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])
                k = (R + f32(0.2)) / ln
                rc = gc + v * k
                out.append((tuple(rc), f32(0.2), mat))
    out.append(((f32(0.0), f32(1.0), f32(0.0)), f32(1.0), ("dielectric", f32(1.5))))
    out.append(((f32(-4.0), f32(1.0), f32(0.0)), f32(1.0), ("lambert", (f32(0.4), f32(0.2), f32(0.1)))))
    out.append(((f32(4.0), f32(1.0), f32(0.0)), f32(1.0), ("metal", (f32(0.7), f32(0.6), f32(0.5)), f32(0.0))))
    return out


# ------------------------------------------------------------------------------------------------
# camera.rs:132-151 (vertical_fov + look_at + optional focus distance / aperture)
# ------------------------------------------------------------------------------------------------
def _libm_tanf(x: float) -> float:
    import ctypes

    m = ctypes.CDLL("libm.so.6")
    m.tanf.restype = ctypes.c_float
    m.tanf.argtypes = [ctypes.c_float]
    return m.tanf(x)


def camera_build(vfov, aspect, position, target, up=(0, 1, 0), focus_distance=None, aperture=0.0):

    def cross(a, b):
        return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]], np.float32)

    def dot(a, b):
        return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]

    def length(a):
        return np.sqrt(dot(a, a))

    def with_length(a, n):
        return a * (f32(n) / length(a))

    rad = f32(vfov) * (f32(3.14159265358979) / f32(180.0))
    h = f32(_libm_tanf(float(f32(rad * f32(0.5)))))  # Rust f32::tan -> the platform tanf
    vw = f32(2.0) * h
    vh = f32(2.0) * h * f32(aspect)
    pos = np.asarray(position, np.float32)
    fwd = np.asarray(target, np.float32) - pos
    upv = np.asarray(up, np.float32)
    fd = f32(1.0) if focus_distance is None else f32(focus_distance)
    ur = with_length(cross(fwd, upv), 1.0)
    uu = with_length(cross(ur, fwd), 1.0)
    sf = with_length(fwd, fd)
    ulc = (ur * (vw * f32(-0.5)) + uu * (vh * f32(0.5))) * fd + sf
    return dict(
        position=pos,
        upper_left_corner=ulc,
        unit_right=ur,
        unit_up=uu,
        scaled_right=ur * (fd * vw),
        scaled_up=uu * (fd * vh),
        lens_radius=f32(aperture) / f32(2.0),
    )
