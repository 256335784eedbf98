"""ctypes binding of librtw.so (include/rtw.h).

The library is built in-tree by ``__graft_entry__.build()`` (raytracinginaweekend_amd/csrc/Makefile)
and loaded from the package directory.  There is no fallback: if the HIP library is missing,
importing anything that renders raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RTW_LIBRARY") or os.path.join(_HERE, "librtw.so")  # override: experiments only

RTW_OK = 0
RTW_ERR_INVALID_ARGUMENT = 1
RTW_ERR_NO_DEVICE = 2
RTW_ERR_HIP = 3
RTW_ERR_OUT_OF_MEMORY = 4
RTW_ERR_UNSUPPORTED = 5
RTW_ERR_IO = 6
RTW_ERR_PARSE = 7

GEOM_SPHERE, GEOM_RECT, GEOM_BOX, GEOM_TRIANGLE = 0, 1, 2, 3
PLANE_XY, PLANE_XZ, PLANE_YZ = 0, 1, 2
MAT_LAMBERT, MAT_METAL, MAT_DIELECTRIC, MAT_DIFFUSE_LIGHT, MAT_ISOTROPIC = 0, 1, 2, 3, 4
TEX_SOLID, TEX_CHECKER, TEX_MARBLE, TEX_IMAGE = 0, 1, 2, 3
BG_SKY, BG_SOLID = 0, 1
MODE_DEFAULT, MODE_NORMALS = 0, 1
LEAF_VOLUME, LEAF_TRANSFORM, LEAF_ANIMATION = 1, 2, 4
LAYOUT_IMAGE, LAYOUT_TILES = 0, 1

F3 = C.c_float * 3
F2 = C.c_float * 2


class BvhNode(C.Structure):
    _fields_ = [("min", F3), ("max", F3), ("axis", C.c_int32), ("left", C.c_int32), ("right", C.c_int32)]


class Leaf(C.Structure):
    _fields_ = [
        ("geom_kind", C.c_int32),
        ("geom_index", C.c_int32),
        ("material", C.c_int32),
        ("flags", C.c_uint32),
        ("neg_inv_density", C.c_float),
        ("offset", F3),
        ("y_sin", C.c_float),
        ("y_cos", C.c_float),
        ("velocity", F3),
    ]


class Sphere(C.Structure):
    _fields_ = [("center", F3), ("radius", C.c_float)]


class Rect(C.Structure):
    _fields_ = [("plane", C.c_int32), ("dist", C.c_float), ("r0", F2), ("r1", F2)]


class Box(C.Structure):
    _fields_ = [("min", F3), ("max", F3)]


class Triangle(C.Structure):
    _fields_ = [("positions", F3 * 3), ("normals", F3 * 3), ("uvs", F2 * 3)]


class Material(C.Structure):
    _fields_ = [("kind", C.c_int32), ("texture", C.c_int32), ("fuzz", C.c_float), ("index_of_refraction", C.c_float)]


class Texture(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("color", F3),
        ("inv_frequency", C.c_float),
        ("even", C.c_int32),
        ("odd", C.c_int32),
        ("scale", C.c_float),
        ("perlin", C.c_int32),
        ("image", C.c_int32),
    ]


class Image(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("rgb", C.POINTER(C.c_uint8))]


class Perlin(C.Structure):
    _fields_ = [
        ("bits", C.c_int32),
        ("ranvec", F3 * 256),
        ("perm_x", C.c_uint32 * 256),
        ("perm_y", C.c_uint32 * 256),
        ("perm_z", C.c_uint32 * 256),
    ]


class Camera(C.Structure):
    _fields_ = [
        ("position", F3),
        ("upper_left_corner", F3),
        ("unit_right", F3),
        ("unit_up", F3),
        ("scaled_right", F3),
        ("scaled_up", F3),
        ("lens_radius", C.c_float),
        ("time0", C.c_float),
        ("time1", C.c_float),
        ("shutter_pace", F2),
    ]


class Background(C.Structure):
    _fields_ = [("kind", C.c_int32), ("color", F3)]


class World(C.Structure):
    _fields_ = [
        ("camera", Camera),
        ("background", Background),
        ("has_light", C.c_int32),
        ("light", Rect),
        ("root", C.c_int32),
        ("node_count", C.c_int32),
        ("nodes", C.POINTER(BvhNode)),
        ("leaf_count", C.c_int32),
        ("leaves", C.POINTER(Leaf)),
        ("sphere_count", C.c_int32),
        ("spheres", C.POINTER(Sphere)),
        ("rect_count", C.c_int32),
        ("rects", C.POINTER(Rect)),
        ("box_count", C.c_int32),
        ("boxes", C.POINTER(Box)),
        ("triangle_count", C.c_int32),
        ("triangles", C.POINTER(Triangle)),
        ("material_count", C.c_int32),
        ("materials", C.POINTER(Material)),
        ("texture_count", C.c_int32),
        ("textures", C.POINTER(Texture)),
        ("image_count", C.c_int32),
        ("images", C.POINTER(Image)),
        ("perlin_count", C.c_int32),
        ("perlins", C.POINTER(Perlin)),
    ]


class RenderParams(C.Structure):
    _fields_ = [
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("samples_per_pixel", C.c_uint32),
        ("max_depth", C.c_int32),
        ("render_mode", C.c_int32),
        ("layout", C.c_int32),
        ("seed", C.c_uint64),
        ("tile_width", C.c_int32),
        ("tile_height", C.c_int32),
        ("part_index", C.c_int32),
        ("part_count", C.c_int32),
        ("thread_count", C.c_int32),
        ("reserved0", C.c_int32),
    ]


class RenderStats(C.Structure):
    _fields_ = [
        (n, C.c_uint64)
        for n in (
            "samples",
            "rays",
            "node_visits",
            "sphere_tests",
            "rect_tests",
            "box_tests",
            "triangle_tests",
            "sphere_hits",
            "rect_hits",
            "box_hits",
            "triangle_hits",
            "material_reads",
            "texel_reads",
        )
    ]

    def as_dict(self) -> dict:
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class CameraSpec(C.Structure):
    _fields_ = [
        ("fov_mode", C.c_int32),
        ("fov_a", C.c_float),
        ("fov_b", C.c_float),
        ("position", F3),
        ("look_mode", C.c_int32),
        ("up", F3),
        ("target", F3),
        ("has_focus_distance", C.c_int32),
        ("focus_distance", C.c_float),
        ("has_focus_point", C.c_int32),
        ("focus_point", F3),
        ("aperture", C.c_float),
        ("time0", C.c_float),
        ("time1", C.c_float),
    ]


class Assets(C.Structure):
    _fields_ = [
        ("suzanne_tris", C.POINTER(C.c_float)),
        ("suzanne_count", C.c_int32),
        ("cube_tris", C.POINTER(C.c_float)),
        ("cube_count", C.c_int32),
        ("earth_rgb", C.POINTER(C.c_uint8)),
        ("earth_width", C.c_int32),
        ("earth_height", C.c_int32),
    ]


PROGRESS_FN = C.CFUNCTYPE(None, C.c_uint64, C.c_uint64, C.c_void_p)  # rtw_progress_fn


class RtwError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"rtw error {code}: {message}")
        self.code = code


ABI_VERSION = 2  # RTW_ABI_VERSION of include/rtw.h
_lib = None

_P = C.c_void_p
_SIGS = {
    "rtw_version": (C.c_int, []),
    "rtw_last_error": (C.c_char_p, []),
    "rtw_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "rtw_render": (C.c_int, [C.POINTER(World), C.POINTER(RenderParams), C.c_int, C.POINTER(C.c_float)]),
    "rtw_world_upload": (C.c_int, [C.POINTER(World), C.c_int, C.POINTER(_P)]),
    "rtw_world_release": (C.c_int, [_P]),
    "rtw_world_tuning": (C.c_int, [_P, C.POINTER(C.c_int)]),
    "rtw_world_kernel": (C.c_int, [_P] + [C.POINTER(C.c_int)] * 4),
    "rtw_world_kernel_name": (C.c_int, [_P, C.c_char_p, C.c_int]),
    "rtw_world_last_frame": (C.c_int, [_P] + [C.POINTER(C.c_int)] * 3),
    "rtw_render_device": (C.c_int, [_P, C.POINTER(RenderParams), _P, _P]),
    "rtw_render_devices": (C.c_int, [C.POINTER(World), C.POINTER(RenderParams), C.POINTER(C.c_int), C.c_int,
                                     C.POINTER(C.c_float)]),
    "rtw_multi_create": (C.c_int, [C.POINTER(World), C.POINTER(C.c_int), C.c_int, C.POINTER(_P)]),
    "rtw_multi_render": (C.c_int, [_P, C.POINTER(RenderParams), _P]),
    "rtw_multi_release": (C.c_int, [_P]),
    "rtw_multi_peer_copies": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "rtw_partition_floats": (C.c_int, [C.POINTER(RenderParams), C.POINTER(C.c_int64)]),
    "rtw_untile_device": (C.c_int, [C.POINTER(RenderParams), _P, C.c_int64, _P, _P]),
    "rtw_render_collect_stats": (C.c_int, [_P, C.POINTER(RenderParams), C.POINTER(RenderStats)]),
    "rtw_render_collect_stats_tree": (C.c_int, [_P, C.POINTER(RenderParams), C.c_int, C.POINTER(RenderStats)]),
    "rtw_render_progress": (C.c_int, [C.POINTER(World), C.POINTER(RenderParams), C.c_int, C.POINTER(C.c_float),
                                      _P, _P]),
    "rtw_render_debug_counters": (
        C.c_int, [_P, C.POINTER(RenderParams), C.POINTER(RenderStats), C.POINTER(C.c_uint64), C.c_int]),
    "rtw_encode_rgb8_device": (C.c_int, [_P, C.c_int64, _P, _P]),
    "rtw_device_eval_scalar": (
        C.c_int,
        [C.c_int, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int64, C.POINTER(C.c_float)],
    ),
    "rtw_device_eval_checker": (C.c_int, [C.c_int, C.POINTER(C.c_float), C.c_int64, C.POINTER(C.c_int32)]),
    "rtw_device_check_division": (
        C.c_int,
        [C.c_int, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)],
    ),
    "rtw_device_eval_node_pass": (
        C.c_int,
        [C.c_int] + [C.POINTER(C.c_float)] * 4 + [C.c_int32, C.c_int64, C.POINTER(C.c_int32)],
    ),
    "rtw_rng_from_seed": (_P, [C.POINTER(C.c_uint8)]),
    "rtw_rng_free": (None, [_P]),
    "rtw_rng_gen_f32": (C.c_float, [_P]),
    "rtw_rng_next_u64": (C.c_uint64, [_P]),
    "rtw_builder_new": (_P, []),
    "rtw_builder_free": (None, [_P]),
    "rtw_texture_solid": (C.c_int32, [_P, C.c_float, C.c_float, C.c_float]),
    "rtw_texture_checker": (C.c_int32, [_P, C.c_float, C.c_int32, C.c_int32]),
    "rtw_texture_marble": (C.c_int32, [_P, C.c_float, _P]),
    "rtw_texture_image_rgb8": (C.c_int32, [_P, C.POINTER(C.c_uint8), C.c_int32, C.c_int32]),
    "rtw_material_lambert": (C.c_int32, [_P, C.c_int32]),
    "rtw_material_metal": (C.c_int32, [_P, C.c_int32, C.c_float]),
    "rtw_material_dielectric": (C.c_int32, [_P, C.c_float]),
    "rtw_material_diffuse_light": (C.c_int32, [_P, C.c_int32]),
    "rtw_material_isotropic": (C.c_int32, [_P, C.c_int32]),
    "rtw_node_group": (C.c_int32, [_P]),
    "rtw_node_sphere": (C.c_int32, [_P, C.c_float, C.c_int32]),
    "rtw_node_rect": (C.c_int32, [_P, C.c_int32, C.POINTER(C.c_float), C.c_float, C.c_float, C.c_int32]),
    "rtw_node_box": (C.c_int32, [_P, C.c_float, C.c_float, C.c_float, C.c_int32]),
    "rtw_node_mesh": (C.c_int32, [_P, C.POINTER(C.c_float), C.c_int32, C.c_int32]),
    "rtw_node_add": (C.c_int, [_P, C.c_int32, C.c_int32]),
    "rtw_node_translate": (C.c_int, [_P, C.c_int32, C.c_float, C.c_float, C.c_float]),
    "rtw_node_rotate_around_up": (C.c_int, [_P, C.c_int32, C.c_float]),
    "rtw_node_animate_moving": (C.c_int, [_P, C.c_int32, C.c_float, C.c_float, C.c_float]),
    "rtw_node_set_all_geo_as_poi": (C.c_int, [_P, C.c_int32]),
    "rtw_node_set_all_geo_density": (C.c_int, [_P, C.c_int32, C.c_float]),
    "rtw_camera_build": (C.c_int, [C.POINTER(CameraSpec), C.POINTER(Camera)]),
    "rtw_camera_aspect_ratio": (C.c_float, [C.POINTER(Camera)]),
    "rtw_builder_finish": (C.c_int, [_P, C.c_int32, C.POINTER(Background), C.POINTER(Camera), C.POINTER(_P)]),
    "rtw_world_get": (C.POINTER(World), [_P]),
    "rtw_world_free": (None, [_P]),
    "rtw_obj_parse": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_int32)]),
    "rtw_free": (None, [_P]),
    "rtw_demo_world": (C.c_int, [C.c_char_p, C.POINTER(Assets), C.POINTER(_P)]),
}


def lib() -> C.CDLL:
    """Load librtw.so (raises if it has not been built: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(the MI355X path has no CPU fallback)"
            )
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if os.environ.get("RTW_LIBRARY") and not hasattr(L, name):
                continue  # an older experiment build (A/B runs only); the product library has them all
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.rtw_version() != ABI_VERSION:
            msg = f"{LIB_PATH} has ABI version {L.rtw_version()}, this package needs {ABI_VERSION}"
            # a mismatched library would read rtw_render_params wrongly: refuse it, unless an A/B run
            # of an older experiment build (RTW_LIBRARY) opts in explicitly
            if not (os.environ.get("RTW_LIBRARY") and os.environ.get("RTW_ALLOW_ABI_MISMATCH") == "1"):
                raise ImportError(msg + ": rebuild it (A/B runs of older builds: RTW_ALLOW_ABI_MISMATCH=1)")
            import warnings

            warnings.warn(msg + " (RTW_ALLOW_ABI_MISMATCH=1): thread_count and later fields are not honoured")
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != RTW_OK:
        msg = lib().rtw_last_error()
        raise RtwError(rc, msg.decode() if msg else "")


def declared_symbols(header_path: str) -> list[str]:
    """Names of every RTW_API function declared in a header (for the export test)."""
    import re

    text = open(header_path).read()
    return re.findall(r"RTW_API\s+[^;{]*?\b(rtw_\w+)\s*\(", text)
