"""Traversal counts of the product kernel's walk (rtw_render_collect_stats_tree, tree 1) on a world's SAH
tree at several spatial-split budgets (RTW_SAH_SPLIT_BUDGET; RTW_SAH_IGNORE_LDS=1 keeps split trees that
leave LDS mode 2), beside the tree's size and the surface-area estimate (rtw_debug_sah_tree), plus the
frame time of each tree (its LDS mode as launched).  Needs a GPU.

python tools/split_stats.py --scene suzanne --budgets 0,0.2,0.5,1 [--time]
"""
import argparse
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="suzanne")
    ap.add_argument("--budgets", default="0.2,0.5,1,2")
    ap.add_argument("--width", type=int, default=480)
    ap.add_argument("--height", type=int, default=270)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--time", action="store_true", help="also time 1080p x 128 frames of each tree")
    a = ap.parse_args()
    import torch

    import raytracinginaweekend_amd as R
    from raytracinginaweekend_amd import _native as N

    fn = N.lib().rtw_debug_sah_tree
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    os.environ["RTW_SAH_IGNORE_LDS"] = "1"
    world = R.demo_world(a.scene)
    for b in a.budgets.split(","):
        os.environ["RTW_SAH_SPLIT_BUDGET"] = b
        out = (C.c_double * 10)()
        N.check(fn(C.cast(world.ptr(), C.c_void_p), out))
        dw = R.DeviceWorld(world, 0)
        st = dw.collect_stats(R.render_params(R.Size2i(a.width, a.height), a.spp, 50, seed=5), tree=1)
        rays = max(1, st["rays"])
        line = (f"{a.scene} budget {b}: nodes {int(out[0])} depth {int(out[1])} | area: node tests {out[2]:.1f} leaf "
                f"tests {out[3]:.1f} | per ray: nodes {st['node_visits'] / rays:.2f} tri {st['triangle_tests'] / rays:.2f} "
                f"sph {st['sphere_tests'] / rays:.2f} rect {st['rect_tests'] / rays:.2f} | rays/sample "
                f"{rays / max(1, st['samples']):.3f}")
        if a.time:
            img = torch.empty(1920 * 1080 * 3, dtype=torch.float32, device="cuda:0")
            p = R.render_params(R.Size2i(1920, 1080), 128, 50, seed=5)
            dw.render_into(p, img.data_ptr(), 0)  # tuning frame
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(2):
                dw.render_into(p, img.data_ptr(), 0)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / 2
            line += f" | 1080p x 128: {dt * 1e3:.1f} ms, {1920 * 1080 * 128 / dt / 1e6:.0f} Msamples/s, {dw.kernel_variant()}"
        print(line, flush=True)
        dw.release()


if __name__ == "__main__":
    main()
