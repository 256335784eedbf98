"""Multi-GPU frame rendering: interleaved tile partition + one collective gather.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Rank r renders the
tiles t with t % N == r of the frame into a compact tile buffer (RTW_LAYOUT_TILES); the buffers
(padded to rank 0's size, rtw_partition_floats) are gathered onto rank 0 (one collective: RCCL's
gather is a group of point-to-point sends to rank 0 over xGMI, W*H*12/N bytes per peer) and rank 0
scatters them into the image (rtw_untile_device).  Only rank 0 holds the gather buffer and the image.  Because the RNG stream is keyed by (seed, pixel, sample), the
image is bit-identical for every N.  PyTorch is plumbing here: device memory, the stream and the
collective; the render itself is librtw.so's kernel.

TileExchange holds the partition arithmetic and the gather/untile step for both device tensors
(RCCL + the untile kernel) and host tensors (gloo + untile_host, the CPU mirror used by the
world-size-2 and -3 tests).  Reference: rendering.rs:222-252 (the reference merges per-thread planes
in one process; here the ranks own disjoint pixels, so the merge is a placement).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

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
    thread_count: int = 1  # the reference's sample-split planes (rendering.rs:222-252)


def tile_slots(size: Size2i, tile: tuple[int, int], part: tuple[int, int]) -> np.ndarray:
    """Pixel index (or -1 for padding) of every slot of one partition's tile buffer (host-side
    mirror of the kernel's layout: owned tiles t = idx, idx + pc, ... row-major inside)."""
    tw, th = tile
    tiles_x = -(-size.width // tw)
    n_tiles = tiles_x * -(-size.height // th)
    idx, pc = part
    owned = np.arange(idx, n_tiles, pc, dtype=np.int64)[:, None]
    j = np.arange(tw * th, dtype=np.int64)[None, :]
    px = (owned % tiles_x) * tw + j % tw
    py = (owned // tiles_x) * th + j // tw
    return np.where((px < size.width) & (py < size.height), py * size.width + px, -1).ravel()


def pack_tiles(image: np.ndarray, size: Size2i, tile: tuple[int, int], part: tuple[int, int], stride: int) -> np.ndarray:
    """A partition's tile buffer (RTW_LAYOUT_TILES, padded to `stride` floats) cut from a full
    (H*W, 3) image: what the kernel writes for that partition."""
    slots = tile_slots(size, tile, part)
    buf = np.zeros(stride, np.float32)
    v = buf[: len(slots) * 3].reshape(-1, 3)
    ok = slots >= 0
    v[ok] = image.reshape(-1, 3)[slots[ok]]
    return buf


def untile_host(gathered: np.ndarray, size: Size2i, tile: tuple[int, int], part_count: int, stride: int) -> np.ndarray:
    """CPU mirror of untile_kernel (rtw_device.hip): the gathered buffers -> (H*W, 3) image."""
    img = np.zeros((size.width * size.height, 3), np.float32)
    for r in range(part_count):
        slots = tile_slots(size, tile, (r, part_count))
        src = gathered[r * stride: r * stride + len(slots) * 3].reshape(-1, 3)
        ok = slots >= 0
        img[slots[ok]] = src[ok]
    return img


class TileExchange:
    """Partition arithmetic + the gather step of one frame for rank `rank` of `world_size`."""

    def __init__(self, spec: FrameSpec, rank: int, world_size: int):
        self.spec, self.rank, self.world_size = spec, rank, world_size
        p0 = render_params(spec.size, 1, 1, tile=spec.tile, part=(0, world_size), layout=N.LAYOUT_TILES)
        self.stride = partition_floats(p0)  # rank 0 owns the most tiles
        self.params = render_params(spec.size, spec.samples_per_pixel, spec.max_depth, seed=spec.seed,
                                    tile=spec.tile, part=(rank, world_size),
                                    layout=N.LAYOUT_TILES if world_size > 1 else N.LAYOUT_IMAGE,
                                    thread_count=spec.thread_count)

    def pixels_this_rank(self) -> int:
        return int((tile_slots(self.spec.size, self.spec.tile, (self.rank, self.world_size)) >= 0).sum())

    def gather(self, tiles, gathered=None) -> None:
        """Gather the padded tile buffers onto rank 0 (RCCL for device tensors, gloo for host ones):
        rank r's buffer lands at gathered[r * stride : (r + 1) * stride] of rank 0's `gathered`;
        other ranks pass None (they send only)."""
        import torch.distributed as dist

        if self.rank == 0:
            parts = list(gathered.view(self.world_size, -1).unbind(0))
            dist.gather(tiles, parts, dst=0)
        else:
            dist.gather(tiles, None, dst=0)

    def untile(self, gathered, image, stream_ptr: int | None = None) -> None:
        """Rank 0: scatter the gathered buffers into the (W*H*3) image."""
        if gathered.is_cuda:
            untile_device(self.params, gathered.data_ptr(), self.stride, image.data_ptr(), stream_ptr)
        else:
            import torch

            img = untile_host(gathered.numpy(), self.spec.size, self.spec.tile, self.world_size, self.stride)
            image.copy_(torch.from_numpy(img.ravel()))


class FrameRenderer:
    """Renders frames of one World on `device` as rank `rank` of `world_size`."""

    def __init__(self, world: World, spec: FrameSpec, rank: int = 0, world_size: int = 1, device: int = 0):
        import torch

        self.torch = torch
        self.spec, self.rank, self.world_size = spec, rank, world_size
        self.dev = torch.device("cuda", device)
        self.dworld = DeviceWorld(world, device)
        self.xchg = TileExchange(spec, rank, world_size)
        self.params = self.xchg.params
        self.stride = self.xchg.stride
        npix = spec.size.width * spec.size.height
        self.image = torch.zeros(npix * 3, dtype=torch.float32, device=self.dev)
        if world_size > 1:
            self.tiles = torch.zeros(self.stride, dtype=torch.float32, device=self.dev)
            self.gathered = (torch.zeros(self.stride * world_size, dtype=torch.float32, device=self.dev)
                             if rank == 0 else None)

    def stream_ptr(self) -> int:
        return self.torch.cuda.current_stream(self.dev).cuda_stream

    def launch(self) -> None:
        """The render kernel alone (asynchronous, on the current stream)."""
        out = self.image if self.world_size == 1 else self.tiles
        self.dworld.render_into(self.params, out.data_ptr(), self.stream_ptr())

    def exchange(self) -> None:
        """One RCCL gather of the tile buffers onto rank 0 + the untile there."""
        if self.world_size == 1:
            return
        self.xchg.gather(self.tiles, self.gathered)
        if self.rank == 0:
            self.xchg.untile(self.gathered, self.image, self.stream_ptr())

    def render_frame(self):
        self.launch()
        self.exchange()
        return self.image

    def pixels_this_rank(self) -> int:
        return self.xchg.pixels_this_rank()
