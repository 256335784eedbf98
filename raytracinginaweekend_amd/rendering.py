"""rendering::render on the MI355X (src/lib/rendering.rs:121-252).

`render` keeps the reference signature.  `thread_count` keeps its meaning for the numbers: the
reference splits each pixel's samples into thread_count planes (split_work_tasks,
rendering.rs:222-237), averages each plane over its own sample count and merges the planes
last-first (merge_planes, rendering.rs:239-252); the device accumulation reproduces exactly that
arithmetic (the parallelism itself is the GPU's, not thread_count threads).  The reference seeds
from entropy (rendering.rs:160); here the seed is explicit.
"""
from __future__ import annotations

import ctypes as C
import enum
from dataclasses import dataclass

import numpy as np

from . import _native as N
from ._native import check, lib
from .world import World


class RenderMode(enum.IntEnum):  # rendering.rs:94-98
    Default = N.MODE_DEFAULT
    Normals = N.MODE_NORMALS


@dataclass(frozen=True)
class Size2i:  # size2i.rs:3-28
    width: int
    height: int

    def count(self) -> int:
        return self.width * self.height

    def aspect_ratio(self) -> float:
        return float(np.float32(self.height) / np.float32(self.width))


DEFAULT_SEED = 0x5EED


def render_params(
    image_size: Size2i,
    samples_per_pixel: int,
    max_depth: int,
    render_mode: RenderMode = RenderMode.Default,
    seed: int = DEFAULT_SEED,
    tile: tuple[int, int] = (8, 8),
    part: tuple[int, int] = (0, 1),
    layout: int = N.LAYOUT_IMAGE,
    thread_count: int = 1,
) -> N.RenderParams:
    if thread_count < 1:  # split_work_tasks divides by thread_count (rendering.rs:223): the reference panics
        raise ValueError("thread_count must be >= 1")
    p = N.RenderParams()
    p.thread_count = thread_count
    p.width, p.height = image_size.width, image_size.height
    p.samples_per_pixel = samples_per_pixel
    p.max_depth = max_depth
    p.render_mode = int(render_mode)
    p.layout = layout
    p.seed = seed
    p.tile_width, p.tile_height = tile
    p.part_index, p.part_count = part
    return p


def render(
    image_size: Size2i,
    thread_count: int,
    samples_per_pixel: int,
    max_depth: int,
    world: World,
    render_mode: RenderMode = RenderMode.Default,
    *,
    seed: int = DEFAULT_SEED,
    device: int = 0,
    progress=None,
) -> np.ndarray:
    """Linear radiance, shape (H*W, 3) f32, row-major from the top-left pixel (Vec<Color>).

    progress: optional callable(done_samples, total_samples), called about every 50 ms while the
    frame renders and once at the end -- the reference's progress thread (rendering.rs:140-157)
    reports the same quantity as a percentage on stderr."""
    p = render_params(image_size, samples_per_pixel, max_depth, render_mode, seed, thread_count=thread_count)
    out = np.zeros((image_size.height * image_size.width, 3), np.float32)
    ptr = out.ctypes.data_as(C.POINTER(C.c_float))
    if progress is None:
        check(lib().rtw_render(world.ptr(), C.byref(p), device, ptr))
    else:
        cb = N.PROGRESS_FN(lambda done, total, _user: progress(int(done), int(total)))
        check(lib().rtw_render_progress(world.ptr(), C.byref(p), device, ptr, C.cast(cb, C.c_void_p), None))
    return out


def render_devices(
    image_size: Size2i,
    thread_count: int,
    samples_per_pixel: int,
    max_depth: int,
    world: World,
    render_mode: RenderMode = RenderMode.Default,
    *,
    devices=(0,),
    seed: int = DEFAULT_SEED,
    tile: tuple[int, int] = (8, 8),
) -> np.ndarray:
    """`render` on several GPUs of one node from one call (rtw_render_devices): entry i of `devices`
    renders the interleaved tiles t % len(devices) == i on its own host thread, the tile buffers meet on
    devices[0] over xGMI.  A device may repeat.  Bit-identical to `render` for every device list."""
    p = render_params(image_size, samples_per_pixel, max_depth, render_mode, seed, tile=tile, thread_count=thread_count)
    p.part_count = 0
    out = np.zeros((image_size.height * image_size.width, 3), np.float32)
    devs = (C.c_int * len(devices))(*devices)
    check(lib().rtw_render_devices(world.ptr(), C.byref(p), devs, len(devices), out.ctypes.data_as(C.POINTER(C.c_float))))
    return out


class MultiDeviceWorld:
    """A World resident on several GPUs (rtw_multi_create): each frame is split over the device list and
    assembled on devices[0] (rtw_multi_render, synchronous)."""

    def __init__(self, world: World, devices):
        self.world = world
        self.devices = list(devices)
        h = C.c_void_p()
        devs = (C.c_int * len(self.devices))(*self.devices)
        check(lib().rtw_multi_create(world.ptr(), devs, len(self.devices), C.byref(h)))
        self._h = h

    def render_into(self, params: N.RenderParams, d_image_ptr: int) -> None:
        """One frame into the W*H*3 f32 device buffer at d_image_ptr (on devices[0])."""
        check(lib().rtw_multi_render(self._h, C.byref(params), C.c_void_p(d_image_ptr)))

    def peer_copies(self) -> int:
        """Tile-buffer copies made with hipMemcpyPeerAsync so far (rtw_multi_peer_copies)."""
        v = C.c_uint64()
        check(lib().rtw_multi_peer_copies(self._h, C.byref(v)))
        return v.value

    def release(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().rtw_multi_release(self._h)
            self._h = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


class DeviceWorld:
    """A World resident in one GPU's HBM (rtw_world_upload), rendered into torch/HIP buffers."""

    def __init__(self, world: World, device: int = 0):
        self.world = world  # keep the host tables alive
        self.device = device
        h = C.c_void_p()
        check(lib().rtw_world_upload(world.ptr(), device, C.byref(h)))
        self._h = h

    def release(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().rtw_world_release(self._h)
            self._h = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass

    def render_into(self, params: N.RenderParams, d_out_ptr: int, stream_ptr: int | None = None) -> None:
        """Asynchronous launch on `stream_ptr` (hipStream_t) into device pointer `d_out_ptr`."""
        check(lib().rtw_render_device(self._h, C.byref(params), C.c_void_p(d_out_ptr), C.c_void_p(stream_ptr or 0)))

    def tuned_trace_min(self) -> int:
        """The dynamic ray-fetch threshold the device settled on (0 while still exploring)."""
        v = C.c_int()
        check(lib().rtw_world_tuning(self._h, C.byref(v)))
        return v.value

    def kernel_variant(self) -> dict:
        """The render-kernel variant of the last render (LDS mode, leaf kinds, texture kinds, tree, and the
        kernel's exact template name)."""
        m, lk, tx, tr = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        check(lib().rtw_world_kernel(self._h, C.byref(m), C.byref(lk), C.byref(tx), C.byref(tr)))
        name = C.create_string_buffer(64)
        check(lib().rtw_world_kernel_name(self._h, name, 64))
        return {"lds_mode": m.value, "leaf_kinds": lk.value, "tex_kinds": tx.value,
                "tree": ("reference", "sah")[tr.value] if tr.value >= 0 else None,
                # the exact template name (GEN included), as rocprofv3's Kernel_Name holds it
                "name": name.value.decode()}

    def last_frame(self) -> dict:
        """The shape of the last frame: render launches, whole-pixel work items (no colour buffer),
        and the dynamic-fetch threshold it ran with (the tuned one once chosen, else the default)."""
        if not hasattr(lib(), "rtw_world_last_frame"):
            # an older experiment build loaded through RTW_LIBRARY (A/B runs): the tuned threshold only
            return {"launches": None, "whole_pixel": None, "trace_min": self.tuned_trace_min()}
        n, wp, tm = C.c_int(), C.c_int(), C.c_int()
        check(lib().rtw_world_last_frame(self._h, C.byref(n), C.byref(wp), C.byref(tm)))
        return {"launches": n.value, "whole_pixel": bool(wp.value == 1), "trace_min": tm.value}

    def collect_stats(self, params: N.RenderParams, tree: int = 0) -> dict:
        """Traversal statistics of one counting-variant render: tree 0 the reference's traversal
        (hittable.rs:429-473), tree 1 the traversal the product kernel runs (the SAH walk, its
        leaf-box proofs and re-traced rays, where the world takes it)."""
        s = N.RenderStats()
        if tree == 0:
            check(lib().rtw_render_collect_stats(self._h, C.byref(params), C.byref(s)))
        else:
            check(lib().rtw_render_collect_stats_tree(self._h, C.byref(params), tree, C.byref(s)))
        return s.as_dict()

    DEBUG_COUNTERS = ("trav_calls", "iters", "node_iters", "leaf_iters", "node_lanes", "leaf_lanes",
                      "alive_lanes", "wait_lanes", "pass_lanes", "sn_iters", "sn_lanes", "sf_iters", "sf_lanes",
                      "shade_calls", "shade_lanes", "trav_cycles", "rest_cycles")

    def debug_counters(self, params: N.RenderParams) -> tuple[dict, dict]:
        """(statistics, wave-level execution counters) of one counting-variant render."""
        s = N.RenderStats()
        c = (C.c_uint64 * len(self.DEBUG_COUNTERS))()
        check(lib().rtw_render_debug_counters(self._h, C.byref(params), C.byref(s), c, len(c)))
        return s.as_dict(), dict(zip(self.DEBUG_COUNTERS, list(c)))


def partition_floats(params: N.RenderParams) -> int:
    n = C.c_int64()
    check(lib().rtw_partition_floats(C.byref(params), C.byref(n)))
    return n.value


def untile_device(params: N.RenderParams, d_tiles: int, stride_floats: int, d_image: int, stream_ptr: int | None = None):
    check(lib().rtw_untile_device(C.byref(params), C.c_void_p(d_tiles), stride_floats, C.c_void_p(d_image),
                                  C.c_void_p(stream_ptr or 0)))


def encode_rgb8_device(d_image: int, pixels: int, d_rgb8: int, stream_ptr: int | None = None) -> None:
    """to_rgb8_gamma2 (color.rs:43-48) on the device: W*H*3 f32 at d_image -> W*H*3 bytes at d_rgb8."""
    check(lib().rtw_encode_rgb8_device(C.c_void_p(d_image), pixels, C.c_void_p(d_rgb8), C.c_void_p(stream_ptr or 0)))


def device_count() -> int:
    n = C.c_int()
    check(lib().rtw_device_count(C.byref(n)))
    return n.value
