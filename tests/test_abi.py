"""The drop-in boundary: librtw.so (the C ABI of include/rtw.h) loads on a host without a GPU,
exports every declared entry point, and its compute entry points fail loudly (no CPU fallback)
when no HIP device is present."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from raytracinginaweekend_amd import _native as N

import raytracinginaweekend_amd as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rtw.h")


def _has_gpu() -> bool:
    n = C.c_int(0)
    N.lib().rtw_device_count(C.byref(n))
    return n.value > 0


def test_library_exports_every_declared_symbol():
    names = N.declared_symbols(HEADER)
    assert len(names) >= 40
    lib = C.CDLL(N.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the dynamic symbol table agrees (no C++ mangling on the boundary)
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert set(names) <= exported


def test_header_compiles_as_c():
    src = '#include "rtw.h"\n#include "rtw_scalar.h"\n#include "rtw_cull.h"\nint main(void){return rtw_version() < 0;}\n'
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-Wno-unused-function", "-fsyntax-only", "-I",
                    os.path.join(ROOT, "include"), "-x", "c", "-"], input=src, text=True, check=True)


def test_version_and_errors():
    assert N.lib().rtw_version() >= 1
    rc = N.lib().rtw_world_upload(None, 0, None)
    assert rc == N.RTW_ERR_INVALID_ARGUMENT
    assert b"null" in N.lib().rtw_last_error()


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU behaviour")
def test_render_without_gpu_fails_loudly():
    world = R.demo_world("final_scene1")
    with pytest.raises(N.RtwError) as e:
        R.render(R.Size2i(8, 8), 1, 1, 5, world)
    assert e.value.code == N.RTW_ERR_NO_DEVICE
    assert "GPU" in str(e.value)


def test_partition_floats_host_side():
    p = R.render_params(R.Size2i(20, 12), 1, 1, tile=(8, 8), part=(1, 3))
    n = C.c_int64()
    assert N.lib().rtw_partition_floats(C.byref(p), C.byref(n)) == 0
    from raytracinginaweekend_amd.distributed import tile_slots

    assert n.value == len(tile_slots(R.Size2i(20, 12), (8, 8), (1, 3))) * 3


def test_render_devices_arguments():
    """rtw_render_devices / rtw_multi_create reject bad device lists before touching a GPU, and without a
    GPU they fail loudly (no CPU fallback)."""
    world = R.demo_world("final_scene1")
    p = R.render_params(R.Size2i(16, 8), 1, 5)
    out = np.zeros((16 * 8, 3), np.float32)
    optr = out.ctypes.data_as(C.POINTER(C.c_float))
    devs = (C.c_int * 2)(0, 0)
    assert N.lib().rtw_render_devices(world.ptr(), C.byref(p), None, 2, optr) == N.RTW_ERR_INVALID_ARGUMENT
    assert N.lib().rtw_render_devices(world.ptr(), C.byref(p), devs, 0, optr) == N.RTW_ERR_INVALID_ARGUMENT
    assert N.lib().rtw_render_devices(world.ptr(), C.byref(p), devs, 2, None) == N.RTW_ERR_INVALID_ARGUMENT
    h = C.c_void_p()
    assert N.lib().rtw_multi_create(None, devs, 2, C.byref(h)) == N.RTW_ERR_INVALID_ARGUMENT
    assert N.lib().rtw_multi_render(None, C.byref(p), None) == N.RTW_ERR_INVALID_ARGUMENT
    assert N.lib().rtw_multi_release(None) == N.RTW_OK
    if not _has_gpu():
        with pytest.raises(N.RtwError) as e:
            R.render_devices(R.Size2i(16, 8), 1, 1, 5, world, devices=(0, 0))
        assert e.value.code == N.RTW_ERR_NO_DEVICE
    bad = (C.c_int * 1)(-1)
    rc = N.lib().rtw_render_devices(world.ptr(), C.byref(p), bad, 1, optr)
    assert rc in (N.RTW_ERR_INVALID_ARGUMENT, N.RTW_ERR_NO_DEVICE)
