"""rtw_render_devices / rtw_multi_*: one caller renders on a list of devices (one call may
use several devices).  On the one-GPU box the list repeats device 0 -- several partitions on one GPU, each
with its own host thread, stream and resident world -- which runs the same partition and untile code as
distinct devices; with RTW_MULTI_FORCE_PEER=1 the tile buffers also take the hipMemcpyPeerAsync copy that
distinct devices take (a same-device peer copy; rtw_multi_peer_copies counts them).  Lists of distinct
devices run where the box has them (test_distinct_devices_*, skipped on one GPU).  Bit-identical to
rtw_render and to the oracle."""
import numpy as np
import pytest

import raytracinginaweekend_amd as R
from oracle import pyoracle as O
from tests.parity import assert_bit_identical

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("peer", [False, True], ids=["d2d", "peer"])
@pytest.mark.parametrize("devices", [(0,), (0, 0), (0, 0, 0), (0, 0, 0, 0, 0, 0, 0, 0)],
                         ids=["1", "2", "3", "8"])
def test_render_devices_bit_identical(worlds, devices, peer, monkeypatch):
    if peer:
        monkeypatch.setenv("RTW_MULTI_FORCE_PEER", "1")
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


@pytest.mark.parametrize("peer", [False, True], ids=["d2d", "peer"])
def test_multi_world_resident_frames(worlds, peer, monkeypatch):
    """The resident form: several frames of one MultiDeviceWorld (the later ones in cost order) at a
    GPU-filling size, each equal to the one-call render; a second tile size in between.  peer: every
    partition's copy goes through hipMemcpyPeerAsync (RTW_MULTI_FORCE_PEER=1), counted."""
    import torch

    if peer:
        monkeypatch.setenv("RTW_MULTI_FORCE_PEER", "1")
    world = worlds("suzanne")
    size = R.Size2i(480, 270)
    ref = R.render(size, 1, 4, 50, world, seed=23)
    mw = R.MultiDeviceWorld(world, (0, 0, 0, 0))
    img = torch.empty(size.count() * 3, dtype=torch.float32, device="cuda:0")
    tiles = [(8, 8), (8, 8), (16, 4), (8, 8)]
    for tile in tiles:
        img.fill_(np.nan)
        mw.render_into(R.render_params(size, 4, 50, seed=23, tile=tile, part=(0, 0)), img.data_ptr())
        assert_bit_identical(img.cpu().numpy().reshape(-1, 3), ref, f"resident 4 partitions, tile {tile}")
    # the peer branch ran for every partition of every frame (and never without the switch)
    assert mw.peer_copies() == (4 * len(tiles) if peer else 0)
    mw.release()


def _distinct_devices(n):
    import torch

    if torch.cuda.device_count() < n:
        pytest.skip(f"needs {n} GPUs (this box has {torch.cuda.device_count()})")


@pytest.mark.parametrize("devices", [(0, 1), (1, 0), (1, 1, 0)], ids=["0-1", "1-0", "1-1-0"])
def test_distinct_devices_bit_identical(worlds, devices):
    """Distinct GPUs: peer access enabled at create, tile buffers copied over xGMI with
    hipMemcpyPeerAsync into devices[0], untiled there; the image equals the one-GPU render."""
    _distinct_devices(2)
    world = worlds("final_scene1")
    size = R.Size2i(100, 56)
    one = R.render(size, 1, 6, 50, world, seed=13)
    assert_bit_identical(R.render_devices(size, 1, 6, 50, world, devices=devices, seed=13), one,
                         f"rtw_render_devices {devices}")


@pytest.mark.parametrize("devices", [(1, 0), (0, 1, 1)], ids=["1-0", "0-1-1"])
def test_distinct_devices_resident(worlds, devices):
    """The resident form on distinct GPUs, the image buffer on cuda:devices[0]; every partition on a
    device other than devices[0] counts one peer copy per frame."""
    import torch

    _distinct_devices(2)
    world = worlds("suzanne")
    size = R.Size2i(240, 135)
    ref = R.render(size, 1, 4, 50, world, seed=29)
    mw = R.MultiDeviceWorld(world, devices)
    img = torch.empty(size.count() * 3, dtype=torch.float32, device=f"cuda:{devices[0]}")
    for _ in range(2):
        img.fill_(np.nan)
        mw.render_into(R.render_params(size, 4, 50, seed=29, part=(0, 0)), img.data_ptr())
        torch.cuda.synchronize(img.device)
        assert_bit_identical(img.cpu().numpy().reshape(-1, 3), ref, f"resident {devices}")
    assert mw.peer_copies() == 2 * sum(d != devices[0] for d in devices)
    mw.release()
