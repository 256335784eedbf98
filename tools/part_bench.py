"""Per-rank frame of an N-GPU split, on one GPU: how fast one rank renders its interleaved tiles
(launch only, no gather) and which dynamic-fetch threshold it tunes.  Estimates the driver's
N-GPU bench (aggregate ~ N x the slowest rank's rate) without N GPUs.

python tools/part_bench.py [--scene final_scene1] [--parts 1,2,4,8] [--ranks ends|all] [--steps 3]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="final_scene1")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=512)
    ap.add_argument("--parts", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--max-depth", type=int, default=50)
    ap.add_argument("--ranks", default="ends", help="'ends' (0 and N-1) or 'all'")
    ap.add_argument("--tile", default="8x8", help="partition tile WxH")
    a = ap.parse_args()
    import torch

    import raytracinginaweekend_amd as R
    from raytracinginaweekend_amd.distributed import FrameRenderer, FrameSpec

    world = R.demo_world(a.scene)
    spec = FrameSpec(R.Size2i(a.width, a.height), a.spp, a.max_depth, 0x5EED,
                     tile=tuple(int(x) for x in a.tile.lower().split("x")))
    for n in [int(x) for x in a.parts.split(",")]:
        for rank in (range(n) if a.ranks == "all" else sorted({0, n - 1})):
            fr = FrameRenderer(world, spec, rank, n, 0)
            fr.launch()  # warm-up frame (tunes the threshold when the frame has room)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(a.steps):
                fr.launch()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / a.steps
            samples = fr.pixels_this_rank() * a.spp
            print(f"{a.scene} tile={a.tile} spp={a.spp} depth={a.max_depth} N={n} rank={rank}: {dt * 1e3:.1f} ms/frame, {samples / dt / 1e6:.1f} Msamples/s per rank, "
                  f"x{n} = {n * samples / dt / 1e6:.0f}, trace_min {fr.dworld.tuned_trace_min()}", flush=True)
            del fr
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
