"""The multi-GPU data path on the CPU: world-size-2 (and 3) gloo process groups run
TileExchange -- the same partition arithmetic, padded gather onto rank 0 and untile as the RCCL path,
with host tensors -- over partition buffers the oracle renders, and rank 0 must reassemble the
single-process oracle frame bit for bit (the image is independent of N)."""
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world_size, port, out_path, scene, size, spp):
    import sys

    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import raytracinginaweekend_amd as R
    from oracle import pyoracle as O
    from raytracinginaweekend_amd.distributed import FrameSpec, TileExchange, pack_tiles

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world_size)
    try:
        spec = FrameSpec(R.Size2i(*size), spp, 50, seed=99)
        x = TileExchange(spec, rank, world_size)
        world = R.demo_world(scene)
        # this rank's partition: the oracle honours the tile partition in image layout
        p = R.render_params(spec.size, spp, 50, seed=99, tile=spec.tile, part=(rank, world_size))
        part_img = O.render(world, p, O.RNG_CTR, 2)
        tiles = torch.from_numpy(pack_tiles(part_img, spec.size, spec.tile, (rank, world_size), x.stride))
        gathered = torch.zeros(x.stride * world_size, dtype=torch.float32) if rank == 0 else None
        x.gather(tiles, gathered)
        if rank == 0:
            image = torch.zeros(spec.size.width * spec.size.height * 3, dtype=torch.float32)
            x.untile(gathered, image)
            np.save(out_path, image.numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world_size,scene,size,spp", [(2, "final_scene1", (44, 26), 3), (3, "cornell_cube", (30, 30), 2)])
def test_gloo_tile_gather_reassembles_the_frame(tmp_path, world_size, scene, size, spp):
    import torch.multiprocessing as mp

    import raytracinginaweekend_amd as R
    from oracle import pyoracle as O
    from tests.parity import assert_bit_identical

    out = str(tmp_path / "img.npy")
    mp.start_processes(_worker, args=(world_size, _free_port(), out, scene, size, spp), nprocs=world_size,
                       start_method="spawn", join=True)
    got = np.load(out).reshape(-1, 3)
    p = R.render_params(R.Size2i(*size), spp, 50, seed=99)
    assert_bit_identical(got, O.render(R.demo_world(scene), p, O.RNG_CTR, 4), "gathered frame")


def test_partition_covers_every_pixel_once():
    import raytracinginaweekend_amd as R
    from raytracinginaweekend_amd.distributed import tile_slots

    size = R.Size2i(37, 21)
    for n in (1, 2, 3, 4, 8):
        seen = np.concatenate([tile_slots(size, (8, 8), (r, n)) for r in range(n)])
        seen = np.sort(seen[seen >= 0])
        assert np.array_equal(seen, np.arange(size.width * size.height))
