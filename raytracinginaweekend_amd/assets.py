"""Scene assets: the reference's input/ files, pre-converted (tools/make_assets.py).

* meshes.npz: cube / suzanne as parsed by rtw_obj_parse (obj_loader.rs, fan quirk included),
  (n, 24) f32 records.  The .obj text itself is not shipped; the parser is tested on CPU.
* earthmap.png: earthmap.jpg decoded by Pillow (libjpeg-turbo).  The reference decodes with
  jpeg-decoder 0.2.6, which may differ by about 1-2 LSB per channel.
"""
from __future__ import annotations

import os

import numpy as np

from .world import AssetSet

ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")
_cache: AssetSet | None = None


def load_assets() -> AssetSet:
    global _cache
    if _cache is None:
        m = np.load(os.path.join(ASSET_DIR, "meshes.npz"), allow_pickle=False)
        from PIL import Image

        earth = np.asarray(Image.open(os.path.join(ASSET_DIR, "earthmap.png")).convert("RGB"), np.uint8)
        _cache = AssetSet(suzanne=m["suzanne"], cube=m["cube"], earth=earth)
    return _cache
