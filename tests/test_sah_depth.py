"""The split SAH tree's depth cap (rtw_sah.cpp SplitBuilder::depth_cap, build_sah_tables), host only.

suzanne's budget-1 split tree is 21 levels deep uncapped; its 16-bit traversal stack (2 B x depth x 1024
lanes) then keeps the world out of LDS mode 2.  build_sah_tables rebuilds it under the largest cap that
lets the nodes, the triangle records and the stack share the 160 KB (lds_mode2_bytes).  The image never
depends on the tree (the GPU tests check the bits), so these tests check the shapes only.
"""
import ctypes as C

import pytest

import raytracinginaweekend_amd as R
from raytracinginaweekend_amd import _native as N


def _tree(world, monkeypatch, cap=None):
    if cap is None:
        monkeypatch.delenv("RTW_SAH_DEPTH_CAP", raising=False)
    else:
        monkeypatch.setenv("RTW_SAH_DEPTH_CAP", str(cap))
    fn = N.lib().rtw_debug_sah_tree
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    out = (C.c_double * 10)()
    N.check(fn(C.cast(world.ptr(), C.c_void_p), out))
    return {"nodes": int(out[0]), "depth": int(out[1]), "node_tests": out[2], "leaf_tests": out[3]}


@pytest.fixture(scope="module")
def suzanne():
    return R.demo_world("suzanne")


def test_auto_cap_fits_mode2(suzanne, monkeypatch):
    free = _tree(suzanne, monkeypatch, cap=0)  # 0: no cap (audits)
    auto = _tree(suzanne, monkeypatch)
    assert free["depth"] > 16 and auto["depth"] <= 16, (free, auto)
    # the mode-2 budget of launch_render: nodes, cull constants, the one leaf record past the mesh's
    # triangle prefix, 968 triangle records, the 16-bit stack, the drain's mailbox
    need = (2 * auto["nodes"] + 1 + (auto["nodes"] + 1) // 2 + 4 * 968) * 16 + auto["depth"] * 1024 * 2 + 36 * 4
    assert need <= 160 * 1024, need
    # the cap costs little: node and leaf tests per ray (surface-area estimate) within 3 %
    assert auto["node_tests"] <= 1.03 * free["node_tests"] and auto["leaf_tests"] <= 1.03 * free["leaf_tests"]


@pytest.mark.parametrize("cap", [11, 13, 18])
def test_forced_caps_hold(suzanne, monkeypatch, cap):
    t = _tree(suzanne, monkeypatch, cap=cap)
    assert t["depth"] <= cap, t


def test_cap_below_the_leaf_count_is_ignored(suzanne, monkeypatch):
    # 969 leaves need 10 levels at least: a cap of 9 cannot hold and the builder runs uncapped
    assert _tree(suzanne, monkeypatch, cap=9)["depth"] == _tree(suzanne, monkeypatch, cap=0)["depth"]
