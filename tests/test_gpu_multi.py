"""rtw_render_devices / rtw_multi_*: one caller renders on a list of devices (one call may
use several devices).  On the one-GPU box the list repeats device 0 -- several partitions on one GPU, each
with its own host thread, stream and resident world -- which runs the same partition, peer-copy and untile
code as distinct devices.  Bit-identical to rtw_render and to the oracle."""
import numpy as np
import pytest

import raytracinginaweekend_amd as R
from oracle import pyoracle as O
from tests.parity import assert_bit_identical

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("devices", [(0,), (0, 0), (0, 0, 0), (0, 0, 0, 0, 0, 0, 0, 0)],
                         ids=["1", "2", "3", "8"])
def test_render_devices_bit_identical(worlds, devices):
    world = worlds("final_scene1")
    size = R.Size2i(100, 56)  # ragged: edge tiles are partial in both axes
    one = R.render(size, 1, 6, 50, world, seed=13)
    many = R.render_devices(size, 1, 6, 50, world, devices=devices, seed=13)
    assert_bit_identical(many, one, f"rtw_render_devices {devices}")


@pytest.mark.parametrize("name", ["suzanne", "cornell_cube", "earth_motion", "final_scene2"])
def test_render_devices_worlds_against_oracle(worlds, name):
    world = worlds(name)
    size = R.Size2i(48, 36)
    img = R.render_devices(size, 1, 4, 50, world, devices=(0, 0, 0), seed=17)
    assert_bit_identical(img, O.render(world, R.render_params(size, 4, 50, seed=17)), f"{name} on 3 partitions")


def test_render_devices_thread_count_and_normals(worlds):
    world = worlds("cornell_box")
    size = R.Size2i(40, 40)
    a = R.render_devices(size, 3, 8, 50, world, devices=(0, 0), seed=19)
    assert_bit_identical(a, R.render(size, 3, 8, 50, world, seed=19), "thread_count 3 on 2 partitions")
    b = R.render_devices(size, 1, 2, 50, world, R.RenderMode.Normals, devices=(0, 0, 0), seed=19)
    assert_bit_identical(b, R.render(size, 1, 2, 50, world, R.RenderMode.Normals, seed=19), "normals, 3 partitions")


def test_multi_world_resident_frames(worlds):
    """The resident form: several frames of one MultiDeviceWorld (the later ones in cost order) at a
    GPU-filling size, each equal to the one-call render; a second tile size in between."""
    import torch

    world = worlds("suzanne")
    size = R.Size2i(480, 270)
    ref = R.render(size, 1, 4, 50, world, seed=23)
    mw = R.MultiDeviceWorld(world, (0, 0, 0, 0))
    img = torch.empty(size.count() * 3, dtype=torch.float32, device="cuda:0")
    for tile in [(8, 8), (8, 8), (16, 4), (8, 8)]:
        img.fill_(np.nan)
        mw.render_into(R.render_params(size, 4, 50, seed=23, tile=tile, part=(0, 0)), img.data_ptr())
        assert_bit_identical(img.cpu().numpy().reshape(-1, 3), ref, f"resident 4 partitions, tile {tile}")
    mw.release()
