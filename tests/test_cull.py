"""The proximity cull (include/rtw_cull.h; DESIGN.md "Proximity cull") is an extra node test the
kernel ANDs with the reference's Aabb::hit_cond.  It must never change a result:

* the error bound behind it holds on a stress set of grazing / sliver / far-origin hits
  (tests/native/cull_bound_check.c);
* the oracle with the cull (RTW_ORACLE_CULL) renders bit-identically to the oracle without it,
  on every demo world, while visiting fewer nodes where the world has cullable leaves.
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import pyoracle as O
from tests.parity import assert_bit_identical

import raytracinginaweekend_amd as R

HERE = os.path.dirname(os.path.abspath(__file__))


def test_cull_error_bound_stress(tmp_path):
    exe = tmp_path / "cbc"
    subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-fno-fast-math", "-o", str(exe),
                    os.path.join(HERE, "native", "cull_bound_check.c"), "-lm"], check=True)
    out = subprocess.run([str(exe), "1500000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:]
    assert "violations 0" in out.stdout


CASES = [
    # world, size, spp, expect fewer node visits
    ("final_scene1", (64, 36), 8, True),
    ("final_scene2", (48, 48), 4, True),
    ("suzanne", (64, 36), 8, True),
    ("cornell_cube", (40, 40), 8, True),
    ("cornell_box", (40, 40), 8, False),
    ("cornell_box_smoke", (40, 40), 4, False),
    ("earth_motion", (36, 64), 4, False),
    ("moving_spheres", (64, 36), 4, False),
    ("perlin_spheres", (64, 36), 4, False),
    ("defocus_blur", (64, 36), 4, False),
]


@pytest.mark.parametrize("name,size,spp,fewer", CASES, ids=[c[0] for c in CASES])
def test_culled_oracle_is_bit_identical(worlds, name, size, spp, fewer):
    w = worlds(name)
    p = R.render_params(R.Size2i(*size), spp, 50, seed=2024)
    ref, st_ref = O.render(w, p, O.RNG_CTR, 8, stats=True)
    cul, st_cul = O.render(w, p, O.RNG_CTR | O.CULL, 8, stats=True)
    assert_bit_identical(cul, ref)
    for k in ("samples", "rays", "sphere_hits", "rect_hits", "box_hits", "triangle_hits", "material_reads",
              "texel_reads"):
        assert st_cul[k] == st_ref[k], k
    assert st_cul["node_visits"] <= st_ref["node_visits"]
    if fewer:
        assert st_cul["node_visits"] < 0.95 * st_ref["node_visits"]


def test_culled_oracle_ref_mode_bit_identical(worlds):
    """The cull is traversal-only: the reference's own RNG scheme (ref mode) is unchanged too."""
    w = worlds("final_scene1")
    p = R.render_params(R.Size2i(48, 27), 6, 50, seed=5)
    a = O.render(w, p, O.RNG_REF, 3)
    b = O.render(w, p, O.RNG_REF | O.CULL, 3)
    assert_bit_identical(b, a)
