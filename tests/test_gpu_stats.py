"""The counting variant of the kernel reports exactly the oracle's traversal statistics (the
inputs of the algorithmic-bytes model in bench.py / DESIGN.md): with the proximity cull
(default) those of the oracle's culled mode, with RTW_NO_CULL=1 those of the reference traversal
itself -- and both kernels render the same bits."""
import os

import pytest

import raytracinginaweekend_amd as R
from oracle import pyoracle as O
from tests.parity import assert_bit_identical

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["final_scene1", "cornell_box", "suzanne", "final_scene2", "earth_mapped"])
def test_stats_match_oracle(worlds, name):
    world = worlds(name)
    p = R.render_params(R.Size2i(32, 24), 4, 50, seed=9)
    dw = R.DeviceWorld(world, 0)
    gpu = dw.collect_stats(p)
    _, ref = O.render(world, p, O.RNG_CTR | O.CULL, stats=True)
    assert gpu == ref


def _render_pair(world, size, spp, seed, monkeypatch):
    """(culled, reference-traversal) images through the host C-ABI entry rtw_render."""
    args = (R.Size2i(*size), 1, spp, 50, world)
    culled = R.render(*args, seed=seed)
    monkeypatch.setenv("RTW_NO_CULL", "1")
    try:
        plain = R.render(*args, seed=seed)
    finally:
        monkeypatch.delenv("RTW_NO_CULL")
    return culled, plain


@pytest.mark.parametrize("name", ["final_scene1", "suzanne", "final_scene2"])
def test_uncull_matches_reference_traversal(worlds, name, monkeypatch):
    world = worlds(name)
    p = R.render_params(R.Size2i(40, 24), 4, 50, seed=21)
    monkeypatch.setenv("RTW_NO_CULL", "1")
    dw_u = R.DeviceWorld(world, 0)
    monkeypatch.delenv("RTW_NO_CULL")
    _, ref = O.render(world, p, O.RNG_CTR, stats=True)
    assert dw_u.collect_stats(p) == ref
    culled, plain = _render_pair(world, (40, 24), 4, 21, monkeypatch)
    assert_bit_identical(culled, plain, name)
    assert_bit_identical(culled, O.render(world, p, O.RNG_CTR), name)


@pytest.mark.parametrize("name,size,spp", [("final_scene1", (960, 540), 64), ("suzanne", (960, 540), 64),
                                           ("final_scene2", (480, 480), 64), ("cornell_cube", (400, 400), 64)])
def test_cull_invariance_large(worlds, name, size, spp, monkeypatch):
    """Size-independent property at a large sample count: culled == reference traversal, bitwise."""
    culled, plain = _render_pair(worlds(name), size, spp, 77, monkeypatch)
    assert_bit_identical(culled, plain, name)


@pytest.mark.parametrize("name", ["final_scene1", "suzanne", "cornell_cube"])
def test_kernel_tree_counts(worlds, name):
    """Counting variant of the traversal the product kernel runs (rtw_render_collect_stats_tree 1,
    the input of bench.py's record bytes): the same paths as the reference's traversal -- samples,
    rays, closest hits per primitive kind, material and texel reads equal -- with the SAH walk's own
    node and leaf visits, fewer than the reference tree's on the SAH worlds."""
    import torch

    world = worlds(name)
    p = R.render_params(R.Size2i(48, 32), 4, 50, seed=5)
    dw = R.DeviceWorld(world, 0)
    out = torch.zeros(48 * 32 * 3, dtype=torch.float32, device="cuda:0")
    dw.render_into(p, out.data_ptr(), torch.cuda.current_stream().cuda_stream)  # sets kernel_variant()
    torch.cuda.synchronize()
    ref = dw.collect_stats(p, tree=0)
    own = dw.collect_stats(p, tree=1)
    same = ["samples", "rays", "sphere_hits", "rect_hits", "box_hits", "triangle_hits", "material_reads", "texel_reads"]
    assert {k: own[k] for k in same} == {k: ref[k] for k in same}
    if dw.kernel_variant()["tree"].startswith("sah"):
        assert own["node_visits"] < ref["node_visits"]
    else:
        assert own == ref
