"""Generates tests/golden/libm_f32.npz: input / output vectors of the platform libm's acosf,
atan2f, sinf and logf (glibc 2.35, the libm the reference's f32::acos / atan2 / sin / ln call on
Linux: vec3.rs:242-243, texture.rs:32,50, hittable.rs:328).

Each function gets random inputs over the ranges the render path reaches plus the inputs (out of a
larger random draw) where glibc's result differs from the correctly rounded one, which is where a
restatement that rounds correctly would fail.  Data only: inputs and libm's outputs as f32 bits.

python tests/golden/make_libm_fixture.py
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "libm_f32.npz")


def _libm():
    m = ctypes.CDLL("libm.so.6")
    for n in ("acosf", "sinf", "logf"):
        getattr(m, n).restype = ctypes.c_float
        getattr(m, n).argtypes = [ctypes.c_float]
    m.atan2f.restype = ctypes.c_float
    m.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
    return m


def _apply(fn, *args):
    return np.array([fn(*(float(a[i]) for a in args)) for i in range(len(args[0]))], np.float32)


def _bits(rng, n):
    return rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)


def _with_diffs(got, want, keep_random, keep_diff):
    """indices: the first keep_random draws, plus up to keep_diff where libm != RN(f64)."""
    nan = np.isnan(got) & np.isnan(want)
    diff = np.nonzero((got.view(np.uint32) != want.view(np.uint32)) & ~nan)[0]
    return np.unique(np.concatenate([np.arange(keep_random), diff[:keep_diff]]))


def main() -> None:
    m = _libm()
    rng = np.random.default_rng(20261017)
    out = {}
    with np.errstate(all="ignore"):
        x = np.concatenate([rng.uniform(-1, 1, 400_000), [-1.0, 1.0, 0.0, -0.0, 0.5, -0.5, 1.0000001, -1.0000001]])
        x = x.astype(np.float32)
        g = _apply(m.acosf, x)
        idx = _with_diffs(g, np.arccos(x.astype(np.float64)).astype(np.float32), 15_000, 10_000)
        out["acosf_x"], out["acosf_y"] = x[idx], g[idx]

        yy = np.concatenate([rng.uniform(-1, 1, 300_000), _bits(rng, 50_000)]).astype(np.float32)
        xx = np.concatenate([rng.uniform(-1, 1, 300_000), _bits(rng, 50_000)]).astype(np.float32)
        sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-45, 3.4e38], np.float32)
        yy = np.concatenate([yy, np.repeat(sp, len(sp))])
        xx = np.concatenate([xx, np.tile(sp, len(sp))])
        g = _apply(m.atan2f, yy, xx)
        want = np.arctan2(yy.astype(np.float64), xx.astype(np.float64)).astype(np.float32)
        idx = np.unique(np.concatenate([_with_diffs(g, want, 15_000, 10_000), np.arange(len(yy) - len(sp) ** 2, len(yy))]))
        out["atan2f_y"], out["atan2f_x"], out["atan2f_r"] = yy[idx], xx[idx], g[idx]

        x = np.concatenate([rng.uniform(-10, 10, 150_000), rng.uniform(-4000, 4000, 150_000), _bits(rng, 100_000),
                            [0.0, -0.0, np.pi, 1e-30, 119.99999, 120.0, np.inf, np.nan]]).astype(np.float32)
        g = _apply(m.sinf, x)
        idx = _with_diffs(g, np.sin(x.astype(np.float64)).astype(np.float32), 15_000, 10_000)
        out["sinf_x"], out["sinf_y"] = x[idx], g[idx]

        # gen::<f32>() values (multiples of 2^-24 in [0, 1), hittable.rs:328) and any f32
        x = np.concatenate([rng.integers(0, 2**24, 300_000) * np.float64(2.0**-24), _bits(rng, 50_000),
                            [0.0, 1.0, np.inf, -1.0, 1e-45, 3e38]]).astype(np.float32)
        g = _apply(m.logf, x)
        idx = _with_diffs(g, np.log(x.astype(np.float64)).astype(np.float32), 15_000, 10_000)
        out["logf_x"], out["logf_y"] = x[idx], g[idx]
    np.savez_compressed(OUT, **out)
    for k, v in out.items():
        print(k, v.shape)


if __name__ == "__main__":
    main()
