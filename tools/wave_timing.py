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
    ap.add_argument("--parts", type=int, default=1, help="render one rank's share of an N-way split")
    ap.add_argument("--rank", type=int, default=0)
    a = ap.parse_args()
    import torch

    import raytracinginaweekend_amd as R
    from raytracinginaweekend_amd import _native as N

    fn = N.lib().rtw_debug_wave_times
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(C.c_ulonglong)]
    buf = np.zeros(3 * 8192, np.uint64)
    dw = R.DeviceWorld(R.demo_world(a.scene), 0)
    if a.parts > 1:
        p = R.render_params(R.Size2i(a.width, a.height), a.spp, 50, part=(a.rank, a.parts), layout=N.LAYOUT_TILES)
        from raytracinginaweekend_amd.rendering import partition_floats

        nf = partition_floats(p)
    else:
        p = R.render_params(R.Size2i(a.width, a.height), a.spp, 50)
        nf = a.width * a.height * 3
    out = torch.empty(nf, dtype=torch.float32, device="cuda:0")
    fx = N.lib().rtw_debug_wave_extra
    fx.restype = C.c_int
    fx.argtypes = [C.POINTER(C.c_ulonglong)]
    ext = np.zeros(8 * 8192, np.uint64)
    for i in range(3):  # tuning frame, then steady frames
        if i == 2:
            torch.cuda.synchronize()
            fx(ext.ctypes.data_as(C.POINTER(C.c_ulonglong)))  # reset: count the last frame only
        dw.render_into(p, out.data_ptr(), 0)
    torch.cuda.synchronize()
    fx(ext.ctypes.data_as(C.POINTER(C.c_ulonglong)))
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
    print(f"{a.scene} {a.width}x{a.height}x{a.spp} part {a.rank}/{a.parts}: waves {len(t)}, starts within {st.max():.3f} ms, "
          f"ends (ms) min {q[0]:.2f} p10 {q[1]:.2f} p50 {q[2]:.2f} p90 {q[3]:.2f} p99 {q[4]:.2f} max {q[5]:.2f}; "
          f"queue empty (ms) min {qd[0]:.2f} p50 {qd[1]:.2f} max {qd[2]:.2f}; drain after it p50 {dr[0]:.2f} p90 {dr[1]:.2f} "
          f"p99 {dr[2]:.2f} max {dr[3]:.2f}")
    idx = np.nonzero(buf.reshape(-1, 3)[:, 1] > 0)[0]
    blk = idx // 16  # RTW_BLOCK / 64 waves per block
    ub, inv = np.unique(blk, return_inverse=True)
    bend = np.full(len(ub), -1.0)
    np.maximum.at(bend, inv, en)
    bdry = np.full(len(ub), 1e30)
    np.minimum.at(bdry, inv, dry)
    qb = np.percentile(bend, [0, 10, 50, 90, 99, 100])
    qbd = np.percentile(bend - bdry, [50, 90, 99, 100])
    print(f"  blocks {len(ub)}: last wave ends (ms) min {qb[0]:.2f} p10 {qb[1]:.2f} p50 {qb[2]:.2f} p90 {qb[3]:.2f} "
          f"p99 {qb[4]:.2f} max {qb[5]:.2f}; block drain (its last end - its first dry) p50 {qbd[0]:.2f} p90 {qbd[1]:.2f} "
          f"p99 {qbd[2]:.2f} max {qbd[3]:.2f}")
    e = ext.reshape(-1, 8).astype(np.int64)[: len(buf) // 3]
    e = e[buf.reshape(-1, 3)[:, 1] > 0]
    order = np.argsort(-(en - dry))
    print(f"  after the queue ran dry: busy lanes p50 {np.median(e[:, 0]):.0f}, samples finished total {e[:, 1].sum()} "
          f"(bounces mean {e[:, 2].sum() / max(1, e[:, 1].sum()):.1f}); slowest-draining waves "
          "(drain ms, busy, samples, bounces sum): "
          + "; ".join(f"{(en - dry)[i]:.2f} {e[i, 0]} {e[i, 1]} {e[i, 2]}" for i in order[:8]))
    print(f"  drain per wave (mean): coop rays {e[:, 4].mean():.1f}, reference re-traces {e[:, 5].mean():.1f}, "
          f"ms in re-traces {e[:, 6].mean() / 1e5:.3f}, in the SAH walk {e[:, 7].mean() / 1e5:.3f}, in coop {e[:, 3].mean() / 1e5:.3f}; "
          "slowest waves (coop rays, re-traces, ms re-trace, ms walk, ms coop): "
          + "; ".join(f"{e[i, 4]} {e[i, 5]} {e[i, 6] / 1e5:.2f} {e[i, 7] / 1e5:.2f} {e[i, 3] / 1e5:.2f}" for i in order[:8]))


if __name__ == "__main__":
    main()
