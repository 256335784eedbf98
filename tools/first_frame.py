"""Where a one-shot drop-in render call spends its time (rtw_render: upload, first frame with the
in-frame tuning in chunk-major order, copy back) against the steady frame of a resident world.

python tools/first_frame.py [--scene final_scene1] [--spp 512]
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
    a = ap.parse_args()
    import torch

    import raytracinginaweekend_amd as R

    world = R.demo_world(a.scene)
    size = R.Size2i(a.width, a.height)
    R.render(R.Size2i(64, 36), 1, 4, 50, world)  # runtime / module load out of the timings
    torch.cuda.synchronize()
    t = time.perf_counter()
    R.render(size, 1, a.spp, 50, world)
    one_shot = time.perf_counter() - t
    t = time.perf_counter()
    dw = R.DeviceWorld(world, 0)
    torch.cuda.synchronize()
    upload = time.perf_counter() - t
    p = R.render_params(size, a.spp, 50)
    out = torch.empty(a.width * a.height * 3, dtype=torch.float32, device="cuda:0")
    times = []
    for _ in range(4):
        torch.cuda.synchronize()
        t = time.perf_counter()
        dw.render_into(p, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t)
    samples = a.width * a.height * a.spp
    print(f"{a.scene} {a.width}x{a.height}x{a.spp}: one-shot rtw_render {one_shot * 1e3:.1f} ms "
          f"({samples / one_shot / 1e6:.0f} Msamples/s); resident world: upload {upload * 1e3:.1f} ms, frames "
          + ", ".join(f"{x * 1e3:.1f}" for x in times) + f" ms; trace_min {dw.tuned_trace_min()}", flush=True)


if __name__ == "__main__":
    main()
