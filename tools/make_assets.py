"""Regenerate raytracinginaweekend_amd/assets/ from the reference's input/ directory.

Run in the build container (it reads /root/reference/input).  Meshes are parsed by the
product's own OBJ loader (rtw_obj_parse, obj_loader.rs semantics); the JPEG is decoded by
Pillow and stored losslessly.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from raytracinginaweekend_amd.world import load_obj_mesh  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/input"
OUT = os.path.join(ROOT, "raytracinginaweekend_amd", "assets")


def main():
    os.makedirs(OUT, exist_ok=True)
    meshes = {}
    for name in ("cube", "suzanne"):
        with open(os.path.join(REF, f"{name}.obj"), "rb") as f:
            meshes[name] = load_obj_mesh(f.read())
        print(name, meshes[name].shape)
    np.savez_compressed(os.path.join(OUT, "meshes.npz"), **meshes)
    from PIL import Image

    im = Image.open(os.path.join(REF, "earthmap.jpg")).convert("RGB")
    im.save(os.path.join(OUT, "earthmap.png"), optimize=True)
    print("earthmap", im.size)


if __name__ == "__main__":
    main()
