"""GPU parity at BASELINE's full frame sizes, against the oracle on a sample of the frame's tiles.

The GPU renders the whole frame through rtw_render (the product path: cost-free first frame with
the in-frame tuner, the work queue, multi-launch accumulation).  The oracle renders only the 8x8
tiles of one partition (tile t is rendered iff t % stride == k; ctr-mode RNG streams are keyed by
pixel and sample, so a subset of tiles is exactly the full frame's values there) at the same spp,
and the owned pixels must be bit-identical.  final_scene1 runs the headline config itself
(BASELINE configs[1]: 1920x1080x512, max_depth 50).
"""
import numpy as np
import pytest

import raytracinginaweekend_amd as R
from oracle import pyoracle as O
from tests.parity import assert_bit_identical

pytestmark = pytest.mark.gpu

# name, width, height, spp, tile stride (prime), owned residue: every BASELINE config at its full
# size and sample count (C2, C4 on one GPU, C3, C5 on one GPU: one launch of whole-pixel work items,
# 32 pixels per resident lane)
CASES = [
    ("final_scene1", 1920, 1080, 512, 509, 170),
    ("suzanne", 1920, 1080, 512, 1013, 77),
    ("cornell_cube", 800, 800, 1024, 97, 31),
    ("earth_motion", 3840, 2160, 2048, 1009, 500),
]


def owned_mask(w, h, stride, k, tile=8):
    ys, xs = np.mgrid[0:h, 0:w]
    tiles_x = (w + tile - 1) // tile
    t = (ys // tile) * tiles_x + (xs // tile)
    return ((t % stride) == k).reshape(-1)


@pytest.mark.parametrize("name,w,h,spp,stride,k", CASES, ids=[c[0] for c in CASES])
def test_full_frame_sampled_tiles_bit_exact(worlds, name, w, h, spp, stride, k):
    world = worlds(name)
    size = R.Size2i(w, h)
    gpu = R.render(size, 1, spp, 50, world, seed=0x5EED)
    p = R.render_params(size, spp, 50, seed=0x5EED, part=(k, stride))
    ref = np.full((w * h, 3), np.nan, np.float32)
    O.render(world, p, O.RNG_CTR, threads=16, out=ref)
    m = owned_mask(w, h, stride, k)
    assert m.sum() >= 1500
    assert_bit_identical(gpu[m], ref[m], f"{name} {w}x{h}x{spp}, tiles t % {stride} == {k}")


@pytest.mark.parametrize("threads", [1, 16])
def test_config_c1_every_pixel_bit_exact(worlds, threads):
    """BASELINE configs[0] (C1): final_scene1 at 400x225x64, max_depth 50 (demo_worlds.rs:395-463 at
    the explicit size main.rs:38-41 takes), the whole frame through rtw_render and compared with the
    oracle on EVERY pixel; thread_count 1 and 16 (main.rs:19's available_parallelism on the GPU box:
    the image is the merge_planes of 16 sample planes, rendering.rs:222-252)."""
    world = worlds("final_scene1")
    size = R.Size2i(400, 225)
    gpu = R.render(size, threads, 64, 50, world, seed=0x5EED)
    ref = O.render(world, R.render_params(size, 64, 50, seed=0x5EED, thread_count=threads), O.RNG_CTR, threads=16)
    assert gpu.shape == ref.shape == (400 * 225, 3)
    assert_bit_identical(gpu, ref, f"C1 final_scene1 400x225x64, thread_count {threads}")


def test_full_frame_multi_launch_sampled_tiles(worlds, monkeypatch):
    """The same at 1080p with a colour buffer of ~25 samples per launch: three launches carrying the
    running sum, and the thread_count planes crossing launch boundaries."""
    world = worlds("final_scene1")
    size = R.Size2i(1920, 1080)
    monkeypatch.setenv("RTW_SAMPLE_BUFFER_BYTES", str(25 * 1920 * 1080 * 12))
    for threads in (1, 7):
        gpu = R.render(size, threads, 64, 50, world, seed=99)
        p = R.render_params(size, 64, 50, seed=99, part=(3, 509), thread_count=threads)
        ref = np.full((1920 * 1080, 3), np.nan, np.float32)
        O.render(world, p, O.RNG_CTR, threads=16, out=ref)
        m = owned_mask(1920, 1080, 509, 3)
        assert_bit_identical(gpu[m], ref[m], f"final_scene1 1080p64, 3 launches, thread_count {threads}")


def test_full_frame_4k_many_launches(worlds, monkeypatch):
    """C5 (earth_motion 3840x2160x2048) with a colour buffer of 400 samples per launch: six launches
    carrying the running sum, and (thread_count 7) the plane partials across launch boundaries."""
    world = worlds("earth_motion")
    w, h = 3840, 2160
    size = R.Size2i(w, h)
    monkeypatch.setenv("RTW_SAMPLE_BUFFER_BYTES", str(400 * w * h * 12))
    monkeypatch.setenv("RTW_WHOLE_PIXEL", "0")  # per-sample items (C5 on one GPU takes whole pixels by default)
    for threads in (1, 7):
        gpu = R.render(size, threads, 2048, 50, world, seed=77)
        p = R.render_params(size, 2048, 50, seed=77, part=(11, 2003), thread_count=threads)
        ref = np.full((w * h, 3), np.nan, np.float32)
        O.render(world, p, O.RNG_CTR, threads=16, out=ref)
        m = owned_mask(w, h, 2003, 11)
        assert m.sum() >= 3000
        assert_bit_identical(gpu[m], ref[m], f"earth_motion 4Kx2048, 6 launches, thread_count {threads}")


# the north-star split: C4 and C5 over 8 GPUs, one rank at a time on this GPU
PARTS = [("suzanne", 1920, 1080, 512, (0, 6), 307), ("earth_motion", 3840, 2160, 2048, (2, 7), 211)]


@pytest.mark.parametrize("name,w,h,spp,ranks,p", PARTS, ids=[c[0] for c in PARTS])
def test_partitioned_full_frames_sampled_tiles(worlds, name, w, h, spp, ranks, p):
    """Ranks of an 8-way TileExchange split (RTW_LAYOUT_TILES: the rank's interleaved tiles t % 8 == r,
    the cost-ordered frames after the first) at the full config, each compared with the oracle on a
    sample of its own tiles (t % 8p == r + 8k): the same bits as the one-GPU frame there."""
    import torch

    from raytracinginaweekend_amd.distributed import FrameRenderer, FrameSpec, tile_slots

    world = worlds(name)
    size = R.Size2i(w, h)
    spec = FrameSpec(size, spp, 50, 0x5EED)
    for r in ranks:
        fr = FrameRenderer(world, spec, r, 8, 0)
        fr.launch()  # chunk-major first frame (tuning), then a cost-ordered one
        fr.launch()
        torch.cuda.synchronize()
        buf = fr.tiles.cpu().numpy().reshape(-1, 3)
        slots = tile_slots(size, spec.tile, (r, 8))
        img = np.full((w * h, 3), np.nan, np.float32)
        ok = slots >= 0
        img[slots[ok]] = buf[: len(slots)][ok]
        k = 8 * (p // 3) + r  # one residue of the rank's tiles modulo 8p
        q = R.render_params(size, spp, 50, seed=0x5EED, part=(k, 8 * p))
        ref = np.full((w * h, 3), np.nan, np.float32)
        O.render(world, q, O.RNG_CTR, threads=16, out=ref)
        m = owned_mask(w, h, 8 * p, k)
        assert m.sum() >= 800
        assert_bit_identical(img[m], ref[m], f"{name} {w}x{h}x{spp} rank {r} of 8, tiles t % {8 * p} == {k}")
        del fr
        torch.cuda.empty_cache()
