"""Profiling driver: one render of a demo world through rtw_render (no torch), for rocprofv3.

python tools/prof_render.py --scene final_scene1 --width 1920 --height 1080 --spp 16
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import raytracinginaweekend_amd as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="final_scene1")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--max-depth", type=int, default=50)
    ap.add_argument("--repeat", type=int, default=1)
    a = ap.parse_args()
    world = R.demo_world(a.scene)
    size = R.Size2i(a.width, a.height)
    for _ in range(a.repeat):
        t = time.perf_counter()
        img = R.render(size, 1, a.spp, a.max_depth, world)
        dt = time.perf_counter() - t
        print(f"{a.scene} {a.width}x{a.height}x{a.spp}: {dt*1e3:.1f} ms incl. upload, "
              f"{a.width*a.height*a.spp/dt/1e6:.1f} Msamples/s, mean {img.mean(0)}", flush=True)


if __name__ == "__main__":
    main()
