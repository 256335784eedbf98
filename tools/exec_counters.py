"""Wave-level execution counters of the render kernel (counting variant) for a few worlds.

python tools/exec_counters.py [--scenes final_scene1,suzanne] [--width 480 --height 270 --spp 16]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import raytracinginaweekend_amd as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", default="final_scene1,suzanne,cornell_cube,final_scene2")
    ap.add_argument("--width", type=int, default=480)
    ap.add_argument("--height", type=int, default=270)
    ap.add_argument("--spp", type=int, default=16)
    a = ap.parse_args()
    for name in a.scenes.split(","):
        w = R.demo_world(name)
        dw = R.DeviceWorld(w, 0)
        p = R.render_params(R.Size2i(a.width, a.height), a.spp, 50)
        st, c = dw.debug_counters(p)
        it = max(1, c["iters"])
        print(f"{name}: per sample nodes {st['node_visits']/st['samples']:.1f} "
              f"leaf-steps {c['leaf_lanes']/st['samples']:.1f} rays {st['rays']/st['samples']:.2f} | "
              f"iters/call {c['iters']/max(1,c['trav_calls']):.1f}, lanes/iter node {c['node_lanes']/it:.1f} "
              f"leaf {c['leaf_lanes']/it:.1f}, iters running node path {c['node_iters']/it:.2f} leaf path "
              f"{c['leaf_iters']/it:.2f}, lanes/shade {c['shade_lanes']/max(1,c['shade_calls']):.1f}, "
              f"shade calls/iter {c['shade_calls']/it:.3f}, alive lanes/iter {c['alive_lanes']/it:.1f}, "
              f"waiting lanes/iter {c['wait_lanes']/it:.1f}, passing lanes/iter {c['pass_lanes']/it:.1f}, "
              f"inline near sphere: iters {c['sn_iters']/it:.2f} lanes/exec {c['sn_lanes']/max(1,c['sn_iters']):.1f}, "
              f"cycles/iter {c['trav_cycles']/it:.0f}, cycles/shade round {c['rest_cycles']/max(1,c['shade_calls']):.0f}, "
              f"traversal share {c['trav_cycles']/max(1,c['trav_cycles']+c['rest_cycles']):.2f}", flush=True)


if __name__ == "__main__":
    main()
