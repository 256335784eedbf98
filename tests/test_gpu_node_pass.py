"""The traversal's node step on the device (rtw_device.hip node_pass: Aabb::hit_cond with exact
Markstein quotients, aabb.rs:65-78, AND the proximity cull) against the oracle's plain restatement
(true divisions, Rust minmax, rtw_cull_axis) on random and special-value cases: axis-parallel and
tiny directions, origins on box planes and at zero, flat and point boxes, t ranges ending exactly
on slab quotients, k = inf nodes.  Decisions must agree bit for bit (1 = node visited)."""
import ctypes as C

import numpy as np
import pytest

from raytracinginaweekend_amd import _native as N
from oracle import pyoracle as O

pytestmark = pytest.mark.gpu

F = C.POINTER(C.c_float)
I = C.POINTER(C.c_int32)


def _device(box, ray, rng_, km, mk_world):
    out = np.empty(len(box), np.int32)
    N.check(N.lib().rtw_device_eval_node_pass(0, box.ctypes.data_as(F), ray.ctypes.data_as(F), rng_.ctypes.data_as(F),
                                              km.ctypes.data_as(F), mk_world, len(box), out.ctypes.data_as(I)))
    return out


def _oracle(box, ray, rng_, km):
    out = np.empty(len(box), np.int32)
    assert O.lib().rtw_oracle_node_pass(box.ctypes.data_as(F), ray.ctypes.data_as(F), rng_.ctypes.data_as(F),
                                        km.ctypes.data_as(F), len(box), out.ctypes.data_as(I)) == 0
    return out


def _cases(rng, n, nice):
    f32 = np.float32
    scale = rng.choice([1.0, 10.0, 1000.0, 1e-3], n).astype(f32)
    c = (rng.uniform(-1, 1, (n, 3)) * scale[:, None]).astype(f32)
    half = (np.abs(rng.normal(0, 1, (n, 3))) * scale[:, None] * rng.choice([0.05, 0.5, 2.0], n)[:, None]).astype(f32)
    half[rng.random((n, 3)) < 0.05] = 0  # flat boxes
    lo, hi = (c - half).astype(f32), (c + half).astype(f32)
    o = (rng.uniform(-1, 1, (n, 3)) * scale[:, None] * 2).astype(f32)
    # origins on box planes and at zero
    on = rng.random((n, 3))
    o = np.where(on < 0.08, lo, np.where(on < 0.16, hi, np.where(on < 0.2, f32(0), o))).astype(f32)
    d = rng.normal(0, 1, (n, 3)).astype(f32)
    d /= np.sqrt((d * d).sum(1, keepdims=True)).astype(f32)
    z = rng.random((n, 3))
    d = np.where(z < 0.06, f32(0), np.where(z < 0.08, f32(2.0**-61), np.where(z < 0.1, f32(-(2.0**-60)), d))).astype(f32)
    if not nice:  # coordinates below 2^-60 (the world guard then takes the true-division path)
        t = rng.random((n, 3))
        o = np.where(t < 0.1, f32(1e-30), np.where(t < 0.15, f32(-3e-39), o)).astype(f32)
        lo = np.where(rng.random((n, 3)) < 0.1, f32(2e-25), lo).astype(f32)
    ts = np.full(n, 0.001, f32)
    with np.errstate(all="ignore"):
        qa = ((lo - o) / d).astype(f32)
        qb = ((hi - o) / d).astype(f32)
    ax = rng.integers(0, 3, n)
    pick = rng.random(n)
    te = np.where(pick < 0.3, f32(np.inf), (rng.random(n) * scale * 4).astype(f32))
    te = np.where((pick > 0.6) & (pick < 0.75), qa[np.arange(n), ax], te)
    te = np.where((pick > 0.75) & (pick < 0.85), qb[np.arange(n), ax], te)
    ts = np.where((pick > 0.85) & (pick < 0.9), qa[np.arange(n), ax], ts)
    te = np.where(pick > 0.97, ts, te)
    ok = np.isfinite(te) | np.isposinf(te)
    te = np.where(ok & ~np.isnan(te), te, f32(np.inf)).astype(f32)
    ts = np.where(np.isfinite(ts), ts, f32(0.001)).astype(f32)
    te = np.maximum(te, ts)  # the traversal keeps te >= ts
    k = np.where(rng.random(n) < 0.2, f32(np.inf), (rng.random(n) * 1e-4).astype(f32))
    m = (rng.random(n) * 1e-3 * scale).astype(f32)
    box = np.ascontiguousarray(np.concatenate([lo, hi], 1), np.float32)
    ray = np.ascontiguousarray(np.concatenate([o, d], 1), np.float32)
    rg = np.ascontiguousarray(np.stack([ts, te], 1), np.float32)
    km = np.ascontiguousarray(np.stack([k, m], 1), np.float32)
    return box, ray, rg, km


@pytest.mark.parametrize("nice", [True, False])
def test_node_step_matches_reference_hit_cond_and_cull(nice):
    rng = np.random.default_rng(11 if nice else 12)
    box, ray, rg, km = _cases(rng, 1_000_000, nice)
    want = _oracle(box, ray, rg, km)
    assert 0.05 < want.mean() < 0.95  # both outcomes well represented
    for mk_world in ([1, 0] if nice else [0]):
        got = _device(box, ray, rg, km, mk_world)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (mk_world, bad[:5], box[bad[:3]], ray[bad[:3]], rg[bad[:3]], km[bad[:3]])


def test_sah_node_test_contains_exact_cull():
    """The SAH walk's node test (one-multiply quotients, cull constants widened x17/16 and a 68u D
    term, rtw_device.hip node_pass_cons) passes every node that the cull with exact quotients and
    the plain constants passes, on every ray the SAH walk traces (Markstein-exact rays): DESIGN.md
    §5.5's containment argument, checked on 2 M random and special-value cases; for both forms of the
    delta (mode 2: k Dq + 68u D, round 2's form; mode 3: the product's, k D^2 + 68u D, with the grown
    interval's ends one FMA each)."""
    for seed, mode in ((21, 2), (22, 2), (23, 3), (24, 3)):
        rng = np.random.default_rng(seed)
        box, ray, rg, km = _cases(rng, 1_000_000, True)
        k = km[:, 0]
        km[:, 0] = np.where(np.isinf(k), k, k * np.float32(1e3)).astype(np.float32)  # sphere-like k too
        got = _device(box, ray, rg, km, mode)
        fast = (got & 4) != 0
        sah, exact = (got & 1) != 0, (got & 2) != 0
        assert fast.mean() > 0.5
        assert 0.05 < exact[fast].mean() < 0.95
        bad = np.nonzero(fast & exact & ~sah)[0]
        assert bad.size == 0, (bad[:5], box[bad[:3]], ray[bad[:3]], rg[bad[:3]], km[bad[:3]])
