"""TEST INFRASTRUCTURE: ctypes binding of oracle/build/librtw_oracle.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, as the
checker / the timed CPU baseline.  The product never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from raytracinginaweekend_amd import _native as N

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "librtw_oracle.so")
RNG_CTR, RNG_REF = 0, 1
CULL = 0x100  # OR into rng_mode: the product's proximity cull on top of the reference traversal

_lib = None


class OracleHit(C.Structure):
    _fields_ = [
        ("hit", C.c_int32),
        ("t", C.c_float),
        ("position", C.c_float * 3),
        ("normal", C.c_float * 3),
        ("uv", C.c_float * 2),
        ("front_face", C.c_int32),
        ("material", C.c_int32),
    ]


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.rtw_oracle_render.restype = C.c_int
        L.rtw_oracle_render.argtypes = [C.POINTER(N.World), C.POINTER(N.RenderParams), C.c_int, C.c_int,
                                        C.POINTER(C.c_float), C.POINTER(N.RenderStats)]
        L.rtw_oracle_scene_hit.restype = C.c_int
        L.rtw_oracle_scene_hit.argtypes = [C.POINTER(N.World), C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_float,
                                           C.c_float, C.c_float, C.POINTER(C.c_uint64), C.POINTER(OracleHit)]
        L.rtw_oracle_camera_ray.restype = C.c_int
        L.rtw_oracle_camera_ray.argtypes = [C.POINTER(N.Camera), C.c_float, C.c_float, C.POINTER(C.c_uint64),
                                            C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.rtw_oracle_ray_color.restype = C.c_int
        L.rtw_oracle_ray_color.argtypes = [C.POINTER(N.World), C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_float,
                                           C.c_int32, C.c_int32, C.POINTER(C.c_uint64), C.POINTER(C.c_float)]
        L.rtw_oracle_sample_color.restype = C.c_int
        L.rtw_oracle_sample_color.argtypes = [C.POINTER(N.World), C.POINTER(N.RenderParams), C.c_int32, C.c_int32,
                                              C.c_uint32, C.POINTER(C.c_float)]
        L.rtw_oracle_eval_scalar.restype = C.c_int
        L.rtw_oracle_eval_scalar.argtypes = [C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int64,
                                             C.POINTER(C.c_float)]
        L.rtw_oracle_node_pass.restype = C.c_int
        L.rtw_oracle_node_pass.argtypes = [C.POINTER(C.c_float)] * 4 + [C.c_int64, C.POINTER(C.c_int32)]
        _lib = L
    return _lib


def render(world, params: N.RenderParams, rng_mode: int = RNG_CTR, threads: int = 8,
           out: np.ndarray | None = None, stats: bool = False):
    """Oracle render: (H*W, 3) f32 (pixels outside the owned partition keep `out`'s values)."""
    n = params.width * params.height
    if out is None:
        out = np.zeros((n, 3), np.float32)
    st = N.RenderStats()
    rc = lib().rtw_oracle_render(world.ptr(), C.byref(params), rng_mode, threads,
                                 out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st) if stats else None)
    if rc != 0:
        raise RuntimeError(f"oracle render failed: {rc}")
    return (out, st.as_dict()) if stats else out


def sample_color(world, params: N.RenderParams, x: int, y: int, s: int) -> np.ndarray:
    """The ctr-mode radiance of sample `s` of pixel (x, y) (one term of the per-pixel sum)."""
    out = np.zeros(3, np.float32)
    rc = lib().rtw_oracle_sample_color(world.ptr(), C.byref(params), x, y, s, out.ctypes.data_as(C.POINTER(C.c_float)))
    if rc != 0:
        raise RuntimeError("oracle sample_color failed")
    return out


def scene_hit(world, origin, direction, time=0.0, t_start=0.001, t_end=float("inf"), rng=(1, 2)):
    o = (C.c_float * 3)(*origin)
    d = (C.c_float * 3)(*direction)
    r = (C.c_uint64 * 2)(*rng)
    h = OracleHit()
    rc = lib().rtw_oracle_scene_hit(world.ptr(), o, d, time, t_start, t_end, r, C.byref(h))
    if rc != 0:
        raise RuntimeError("oracle scene_hit failed")
    return h, (r[0], r[1])


def eval_scalar(fn: int, a: np.ndarray, b: np.ndarray | None = None) -> np.ndarray:
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(a if b is None else b, np.float32)
    out = np.empty_like(a)
    f = C.POINTER(C.c_float)
    rc = lib().rtw_oracle_eval_scalar(fn, a.ctypes.data_as(f), b.ctypes.data_as(f), len(a), out.ctypes.data_as(f))
    if rc != 0:
        raise RuntimeError("oracle eval failed")
    return out
