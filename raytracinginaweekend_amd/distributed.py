"""Multi-GPU frame rendering: interleaved tile partition + one RCCL gather.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Rank r renders the
tiles t with t % N == r of the frame into a compact tile buffer (RTW_LAYOUT_TILES); the buffers
(padded to rank 0's size) are all-gathered and rank 0 scatters them into the image with
rtw_untile_device.  Because the RNG stream is keyed by (seed, pixel, sample), the image is
bit-identical for every N.  PyTorch is plumbing here: device memory, the stream and the
collective; the render itself is librtw.so's kernel.
"""
from __future__ import annotations

from dataclasses import dataclass

from . import _native as N
from .rendering import DeviceWorld, Size2i, partition_floats, render_params, untile_device
from .world import World


@dataclass
class FrameSpec:
    size: Size2i
    samples_per_pixel: int
    max_depth: int
    seed: int = 0x5EED
    tile: tuple[int, int] = (8, 8)


def tile_slots(size: Size2i, tile: tuple[int, int], part: tuple[int, int]):
    """Pixel index (or -1 for padding) of every slot of one partition's tile buffer (host-side
    mirror of the kernel's layout, used by the CPU tests of the gather/untile logic)."""
    import numpy as np

    tw, th = tile
    tiles_x = -(-size.width // tw)
    n_tiles = tiles_x * -(-size.height // th)
    idx, pc = part
    owned = np.arange(idx, n_tiles, pc, dtype=np.int64)[:, None]
    j = np.arange(tw * th, dtype=np.int64)[None, :]
    px = (owned % tiles_x) * tw + j % tw
    py = (owned // tiles_x) * th + j // tw
    return np.where((px < size.width) & (py < size.height), py * size.width + px, -1).ravel()


class FrameRenderer:
    """Renders frames of one World on `device` as rank `rank` of `world_size`."""

    def __init__(self, world: World, spec: FrameSpec, rank: int = 0, world_size: int = 1, device: int = 0):
        import torch

        self.torch = torch
        self.spec, self.rank, self.world_size = spec, rank, world_size
        self.dev = torch.device("cuda", device)
        self.dworld = DeviceWorld(world, device)
        layout = N.LAYOUT_TILES if world_size > 1 else N.LAYOUT_IMAGE
        self.params = render_params(spec.size, spec.samples_per_pixel, spec.max_depth, seed=spec.seed,
                                    tile=spec.tile, part=(rank, world_size), layout=layout)
        p0 = render_params(spec.size, 1, 1, tile=spec.tile, part=(0, world_size), layout=N.LAYOUT_TILES)
        self.stride = partition_floats(p0)  # rank 0 owns the most tiles
        npix = spec.size.width * spec.size.height
        self.image = torch.zeros(npix * 3, dtype=torch.float32, device=self.dev)
        if world_size > 1:
            self.tiles = torch.zeros(self.stride, dtype=torch.float32, device=self.dev)
            self.gathered = torch.zeros(self.stride * world_size, dtype=torch.float32, device=self.dev)

    def stream_ptr(self) -> int:
        return self.torch.cuda.current_stream(self.dev).cuda_stream

    def launch(self) -> None:
        """The render kernel alone (asynchronous, on the current stream)."""
        out = self.image if self.world_size == 1 else self.tiles
        self.dworld.render_into(self.params, out.data_ptr(), self.stream_ptr())

    def exchange(self) -> None:
        """One RCCL all-gather of the tile buffers + the untile on rank 0."""
        if self.world_size == 1:
            return
        import torch.distributed as dist

        dist.all_gather_into_tensor(self.gathered, self.tiles)
        if self.rank == 0:
            untile_device(self.params, self.gathered.data_ptr(), self.stride, self.image.data_ptr(), self.stream_ptr())

    def render_frame(self):
        self.launch()
        self.exchange()
        return self.image

    def pixels_this_rank(self) -> int:
        return int((tile_slots(self.spec.size, self.spec.tile, (self.rank, self.world_size)) >= 0).sum())
