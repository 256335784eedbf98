"""thread_count semantics of rendering::render (rendering.rs:161-252), CPU side.

The reference splits each pixel's samples into thread_count planes (split_work_tasks,
rendering.rs:222-237: spp / T each, the first spp % T planes one more, planes of 0 samples
dropped), averages each plane over its own count (`.sum::<Color>() / n as f32`, :172-179) and
merges last-plane-first (merge_planes, :239-252: pop the last, += planes 0..n-2, *= 1/n).  Here
that arithmetic is restated in numpy f32 from the oracle's per-sample radiances and compared bit
for bit with the oracle's ctr-mode render (the device is compared with the same oracle in
tests/test_gpu_parity.py)."""
import numpy as np
import pytest

from oracle import pyoracle as O
from tests.parity import assert_bit_identical

import raytracinginaweekend_amd as R


def split_work_tasks(spp: int, t: int) -> list[int]:
    """rendering.rs:222-237."""
    whole, rem = divmod(spp, t)
    out = []
    for i in range(t):
        n = whole + (1 if i < rem else 0)
        if n == 0:
            break
        out.append(n)
    return out


def merged_pixel(cols: np.ndarray, tasks: list[int]) -> np.ndarray:
    f32 = np.float32
    planes, s = [], 0
    for n in tasks:
        acc = np.zeros(3, f32)
        for _ in range(n):
            acc = (acc + cols[s]).astype(f32)
            s += 1
        planes.append((acc / f32(n)).astype(f32))
    mult = f32(1.0) / f32(len(planes))
    px = planes.pop()
    for p in planes:
        px = (px + p).astype(f32)
    return (px * mult).astype(f32) if len(tasks) > 1 else px


def test_split_work_tasks_shapes():
    assert split_work_tasks(512, 1) == [512]
    assert split_work_tasks(10, 3) == [4, 3, 3]
    assert split_work_tasks(5, 16) == [1, 1, 1, 1, 1]
    assert split_work_tasks(16, 16) == [1] * 16


@pytest.mark.parametrize("threads,spp", [(1, 7), (3, 7), (7, 7), (16, 7), (2, 8)])
def test_oracle_planes_match_numpy_merge(worlds, threads, spp):
    world = worlds("final_scene1")
    size = R.Size2i(5, 4)
    p = R.render_params(size, spp, 50, seed=9, thread_count=threads)
    img = O.render(world, p, O.RNG_CTR, 2)
    tasks = split_work_tasks(spp, threads)
    want = np.zeros_like(img)
    for y in range(size.height):
        for x in range(size.width):
            cols = np.stack([O.sample_color(world, p, x, y, s) for s in range(spp)])
            want[y * size.width + x] = merged_pixel(cols, tasks)
    assert_bit_identical(img, want, f"T={threads}")


def test_thread_count_one_is_the_plain_mean(worlds):
    world = worlds("cornell_box")
    size = R.Size2i(6, 6)
    a = O.render(world, R.render_params(size, 9, 50, seed=2), O.RNG_CTR, 2)
    b = O.render(world, R.render_params(size, 9, 50, seed=2, thread_count=1), O.RNG_CTR, 2)
    assert_bit_identical(a, b, "T=1")


def test_thread_count_zero_rejected():
    with pytest.raises(ValueError):
        R.render_params(R.Size2i(4, 4), 4, 5, thread_count=0)
