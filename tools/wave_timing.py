"""Per-wave start / end times of one render launch (experiment build only):

  make -C raytracinginaweekend_amd/csrc variant V=wt DEFS=-DRTW_WAVE_TIMING
  RTW_LIBRARY=$PWD/raytracinginaweekend_amd/librtw_wt.so python tools/wave_timing.py --scene final_scene1 --spp 64

Prints the launch's span and when the waves finish (ms after the first wave started): how long
the frame's tail is, where the GPU runs out of work wave by wave.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="final_scene1")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    a = ap.parse_args()
    import torch

    import raytracinginaweekend_amd as R
    from raytracinginaweekend_amd import _native as N

    fn = N.lib().rtw_debug_wave_times
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(C.c_ulonglong)]
    buf = np.zeros(3 * 8192, np.uint64)
    dw = R.DeviceWorld(R.demo_world(a.scene), 0)
    p = R.render_params(R.Size2i(a.width, a.height), a.spp, 50)
    out = torch.empty(a.width * a.height * 3, dtype=torch.float32, device="cuda:0")
    for _ in range(3):  # tuning frame, then steady frames
        dw.render_into(p, out.data_ptr(), 0)
    torch.cuda.synchronize()
    if fn(buf.ctypes.data_as(C.POINTER(C.c_ulonglong))) != 0:
        raise SystemExit("library built without RTW_WAVE_TIMING")
    t = buf.reshape(-1, 3).astype(np.int64)
    t = t[t[:, 1] > 0]
    t0 = t[:, 0].min()
    st = (t[:, 0] - t0) / 1e5  # 100 MHz -> ms
    en = (t[:, 1] - t0) / 1e5
    q = np.percentile(en, [0, 10, 50, 90, 99, 100])
    dry = (t[:, 2] - t0) / 1e5
    qd = np.percentile(dry, [0, 50, 100])
    dr = np.percentile(en - dry, [50, 90, 99, 100])
    print(f"{a.scene} {a.width}x{a.height}x{a.spp}: waves {len(t)}, starts within {st.max():.3f} ms, "
          f"ends (ms) min {q[0]:.2f} p10 {q[1]:.2f} p50 {q[2]:.2f} p90 {q[3]:.2f} p99 {q[4]:.2f} max {q[5]:.2f}; "
          f"queue empty (ms) min {qd[0]:.2f} p50 {qd[1]:.2f} max {qd[2]:.2f}; drain after it p50 {dr[0]:.2f} p90 {dr[1]:.2f} "
          f"p99 {dr[2]:.2f} max {dr[3]:.2f}")


if __name__ == "__main__":
    main()
