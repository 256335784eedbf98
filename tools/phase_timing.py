"""Wall-cycle split of the render kernel's main loop (experiment build only):

  make -C raytracinginaweekend_amd/csrc variant V=pt DEFS=-DRTW_PHASE_TIMING
  RTW_LIBRARY=$PWD/raytracinginaweekend_amd/librtw_pt.so python tools/phase_timing.py --scene final_scene1

Phases (per wave, summed over waves; a wave's cycles include the time other waves on its SIMD
issue; the phase is switched by the wave's first active lane, so divergent sub-phases count whole-wave
cycles): 1 refill (work items), 2 traversal setup (the ray's reciprocals), 3 traversal (SAH walk,
drain, proof, re-traces), 4 shading (hit record, material, texture, pdf), 5 sample start (stream
setup, jitter, camera ray and its UnitDisc), 6 shading's samplers (UnitSphere / UnitBall rejection
loops, gen_bool, light direction), 7 colour store and cost bookkeeping.  The frame after a warm-up
frame (cost order, tuned threshold).
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="final_scene1")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=128)
    a = ap.parse_args()
    import torch

    import raytracinginaweekend_amd as R
    from raytracinginaweekend_amd import _native as N

    lib = N.lib()
    fn = lib.rtw_debug_phase_cycles
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(C.c_ulonglong)]
    buf = (C.c_ulonglong * 8)()
    dw = R.DeviceWorld(R.demo_world(a.scene), 0)
    p = R.render_params(R.Size2i(a.width, a.height), a.spp, 50)
    out = torch.empty(a.width * a.height * 3, dtype=torch.float32, device="cuda:0")
    dw.render_into(p, out.data_ptr(), 0)  # warm-up: tuning frame
    torch.cuda.synchronize()
    fn(buf)
    dw.render_into(p, out.data_ptr(), 0)
    torch.cuda.synchronize()
    if fn(buf) != 0:
        raise SystemExit("library built without RTW_PHASE_TIMING")
    names = {1: "refill", 2: "traversal setup", 3: "traversal", 4: "shading", 5: "sample start",
             6: "samplers", 7: "stores"}
    tot = sum(buf[k] for k in names)
    print(a.scene, f"{a.width}x{a.height}x{a.spp}", " ".join(f"{names[k]} {buf[k] / tot:.4f}" for k in names),
          f"(wave cycles {tot})", flush=True)


if __name__ == "__main__":
    main()
