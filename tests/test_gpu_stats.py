"""The counting variant of the kernel reports exactly the oracle's traversal statistics (the
inputs of the algorithmic-bytes model in bench.py / DESIGN.md)."""
import pytest

import raytracinginaweekend_amd as R
from oracle import pyoracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["final_scene1", "cornell_box", "suzanne", "final_scene2", "earth_mapped"])
def test_stats_match_oracle(worlds, name):
    world = worlds(name)
    p = R.render_params(R.Size2i(32, 24), 4, 50, seed=9)
    dw = R.DeviceWorld(world, 0)
    gpu = dw.collect_stats(p)
    _, ref = O.render(world, p, stats=True)
    assert gpu == ref
