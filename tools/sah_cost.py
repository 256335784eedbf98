"""Surface-area cost of the render kernel's SAH tree for a demo world (host only, no GPU):
node count, depth, expected node and leaf tests per ray (rtw_debug_sah_tree), for a list of
spatial-split budgets (RTW_SAH_SPLIT_BUDGET).

python tools/sah_cost.py --scene suzanne --budgets 0,0.1,0.2,0.3
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="suzanne")
    ap.add_argument("--budgets", default="0,0.1,0.2,0.3")
    a = ap.parse_args()
    import raytracinginaweekend_amd as R
    from raytracinginaweekend_amd import _native as N

    fn = N.lib().rtw_debug_sah_tree
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    world = R.demo_world(a.scene)
    for b in a.budgets.split(","):
        os.environ["RTW_SAH_SPLIT_BUDGET"] = b
        out = (C.c_double * 10)()
        N.check(fn(C.cast(world.ptr(), C.c_void_p), out))
        print(f"{a.scene} budget {b}: nodes {int(out[0])} depth {int(out[1])} node tests/ray {out[2]:.2f} "
              f"leaf tests/ray {out[3]:.2f} sah {int(out[4])} | 2-wide steps {out[5]:.2f} box tests {out[6]:.2f} | "
              f"4-wide steps {out[7]:.2f} box tests {out[8]:.2f} leaf tests {out[9]:.2f}", flush=True)


if __name__ == "__main__":
    main()
