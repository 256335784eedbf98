"""Host-side scene construction: the Python face of the reference's Camera / WorldBuilder API.

Mirrors src/lib/camera.rs:11-152 (typestate camera builder), src/app/worlds/world_builder.rs
(WorldBuilder, NodeBuilder, NodeRef::finish) and src/app/worlds/demo_worlds.rs.  The work is
done by the C++ builder in librtw.so (csrc/scene_builder.cpp, csrc/demo_worlds.cpp); these
classes only hold ids and forward calls, raising RtwError where the reference panics.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _native as N
from ._native import check, lib


# ------------------------------------------------------------------------------------------------
# Camera (camera.rs)
# ------------------------------------------------------------------------------------------------
class Camera:
    """A built camera (camera.rs:154-164)."""

    def __init__(self, raw: N.Camera):
        self.raw = raw

    @staticmethod
    def build() -> "CameraBuilder":
        return CameraBuilder()

    def aspect_ratio(self) -> float:  # camera.rs:171-173
        return float(lib().rtw_camera_aspect_ratio(C.byref(self.raw)))

    @property
    def time_interval(self) -> tuple[float, float]:
        return (self.raw.time0, self.raw.time1)


class CameraBuilder:
    """camera.rs:11-152: viewport|vertical_fov -> position -> orientation|look_at|look_at_focus ->
    [focus_point, aperture, focus_distance, motion_blur] -> build."""

    def __init__(self):
        self.s = N.CameraSpec()
        self.s.up[:] = (0.0, 1.0, 0.0)
        self.s.target[:] = (0.0, 0.0, -1.0)  # Dir3::FORWARD
        self._stage = 0

    def _need(self, stage: int, name: str) -> None:
        if self._stage != stage:
            raise TypeError(f"CameraBuilder.{name} called out of order (camera.rs typestate)")

    def viewport(self, width: float, height: float) -> "CameraBuilder":
        self._need(0, "viewport")
        self.s.fov_mode, self.s.fov_a, self.s.fov_b = 0, width, height
        self._stage = 1
        return self

    def vertical_fov(self, vertical_field_of_view: float, aspect_ratio: float) -> "CameraBuilder":
        self._need(0, "vertical_fov")
        self.s.fov_mode, self.s.fov_a, self.s.fov_b = 1, vertical_field_of_view, aspect_ratio
        self._stage = 1
        return self

    def position(self, pos) -> "CameraBuilder":
        self._need(1, "position")
        self.s.position[:] = tuple(pos)
        self._stage = 2
        return self

    def _look(self, mode: int, up, target, name: str) -> "CameraBuilder":
        self._need(2, name)
        self.s.look_mode = mode
        self.s.up[:] = tuple(up)
        self.s.target[:] = tuple(target)
        self._stage = 3
        return self

    def orientation(self, up, forward) -> "CameraBuilder":
        return self._look(0, up, forward, "orientation")

    def look_at(self, up, pos) -> "CameraBuilder":
        return self._look(1, up, pos, "look_at")

    def look_at_focus(self, up, pos) -> "CameraBuilder":
        return self._look(2, up, pos, "look_at_focus")

    def focus_point(self, pos) -> "CameraBuilder":
        self._need(3, "focus_point")
        self.s.has_focus_point = 1
        self.s.focus_point[:] = tuple(pos)
        return self

    def aperture(self, aperture: float) -> "CameraBuilder":
        self._need(3, "aperture")
        self.s.aperture = aperture
        return self

    def focus_distance(self, distance: float) -> "CameraBuilder":
        self._need(3, "focus_distance")
        self.s.has_focus_distance = 1
        self.s.focus_distance = distance
        return self

    def motion_blur(self, start: float, end: float) -> "CameraBuilder":
        self._need(3, "motion_blur")
        self.s.time0, self.s.time1 = start, end
        return self

    def build(self) -> Camera:
        self._need(3, "build")
        cam = N.Camera()
        check(lib().rtw_camera_build(C.byref(self.s), C.byref(cam)))
        return Camera(cam)


# ------------------------------------------------------------------------------------------------
# Background (background_color.rs)
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class BackgroundColor:
    kind: int = N.BG_SKY
    color: tuple = (0.0, 0.0, 0.0)

    @staticmethod
    def sky() -> "BackgroundColor":
        return BackgroundColor(N.BG_SKY)

    @staticmethod
    def solid(color) -> "BackgroundColor":
        return BackgroundColor(N.BG_SOLID, tuple(float(c) for c in color))

    def raw(self) -> N.Background:
        b = N.Background()
        b.kind = self.kind
        b.color[:] = self.color
        return b


# ------------------------------------------------------------------------------------------------
# The finished world (rendering.rs:12-17), owned by the C++ side
# ------------------------------------------------------------------------------------------------
class World:
    """A finished World: camera + one BVH over the flattened leaves + tables (include/rtw.h)."""

    def __init__(self, handle: int):
        self._handle = C.c_void_p(handle)
        self.raw: N.World = lib().rtw_world_get(self._handle).contents

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            try:
                lib().rtw_world_free(h)
            except Exception:
                pass
            self._handle = None

    @property
    def camera(self) -> Camera:
        return Camera(self.raw.camera)

    def ptr(self):
        return C.byref(self.raw)

    # convenience views (copies) for tests
    def nodes(self) -> np.ndarray:
        n = self.raw.node_count
        return np.ctypeslib.as_array(self.raw.nodes, (n,)).copy() if n else np.zeros(0)

    def leaves(self) -> list:
        return [self.raw.leaves[i] for i in range(self.raw.leaf_count)]

    def spheres(self) -> np.ndarray:
        n = self.raw.sphere_count
        out = np.zeros((n, 4), np.float32)
        for i in range(n):
            s = self.raw.spheres[i]
            out[i, :3] = list(s.center)
            out[i, 3] = s.radius
        return out


# ------------------------------------------------------------------------------------------------
# WorldBuilder / NodeBuilder (world_builder.rs)
# ------------------------------------------------------------------------------------------------
def _ok(i: int) -> int:
    if i < 0:
        check(N.RTW_ERR_INVALID_ARGUMENT)
    return i


class Rng:
    """TRng = Xoroshiro128PlusPlus (common.rs:1), seeded from 16 bytes (main.rs:24)."""

    def __init__(self, seed: bytes = bytes(range(1, 17))):
        assert len(seed) == 16
        buf = (C.c_uint8 * 16).from_buffer_copy(seed)
        self._p = C.c_void_p(lib().rtw_rng_from_seed(buf))

    def gen_f32(self) -> float:
        return float(lib().rtw_rng_gen_f32(self._p))

    def next_u64(self) -> int:
        return int(lib().rtw_rng_next_u64(self._p))

    def __del__(self):
        if getattr(self, "_p", None) is not None and self._p.value:
            lib().rtw_rng_free(self._p)
            self._p = None


class NodeRef:
    def __init__(self, wb: "WorldBuilder", nid: int):
        self.wb, self.id = wb, nid

    def finish(self, wb: "WorldBuilder", background: BackgroundColor, camera: Camera) -> World:
        """world_builder.rs:273-290: flatten, one BVH over camera.time_interval."""
        out = C.c_void_p()
        bg = background.raw()
        check(lib().rtw_builder_finish(wb._b, self.id, C.byref(bg), C.byref(camera.raw), C.byref(out)))
        return World(out.value)


class NodeBuilder(NodeRef):
    """world_builder.rs:228-270 (mutating builder; `build()` returns the shared NodeRef)."""

    def add(self, elem: NodeRef) -> "NodeBuilder":
        check(lib().rtw_node_add(self.wb._b, self.id, elem.id))
        return self

    def set_all_geo_as_poi(self) -> "NodeBuilder":
        check(lib().rtw_node_set_all_geo_as_poi(self.wb._b, self.id))
        return self

    def rotate_around_up(self, angle: float) -> "NodeBuilder":
        check(lib().rtw_node_rotate_around_up(self.wb._b, self.id, angle))
        return self

    def translate(self, offset) -> "NodeBuilder":
        x, y, z = offset
        check(lib().rtw_node_translate(self.wb._b, self.id, x, y, z))
        return self

    def animate_moving(self, velocity) -> "NodeBuilder":
        x, y, z = velocity
        check(lib().rtw_node_animate_moving(self.wb._b, self.id, x, y, z))
        return self

    def set_all_geo_densitity(self, densitity: float) -> "NodeBuilder":
        check(lib().rtw_node_set_all_geo_density(self.wb._b, self.id, densitity))
        return self

    def build(self) -> NodeRef:
        return NodeRef(self.wb, self.id)


class WorldBuilder:
    """world_builder.rs:7-192 (textures, materials and geometry-node factories)."""

    def __init__(self):
        self._b = C.c_void_p(lib().rtw_builder_new())

    def __del__(self):
        if getattr(self, "_b", None) is not None and self._b.value:
            lib().rtw_builder_free(self._b)
            self._b = None

    # textures
    def texture_solid(self, color) -> int:
        return _ok(lib().rtw_texture_solid(self._b, *map(float, color)))

    def texture_checker(self, inv_frequency: float, tex_even: int, tex_odd: int) -> int:
        return _ok(lib().rtw_texture_checker(self._b, inv_frequency, tex_even, tex_odd))

    def texture_marble(self, scale: float, rng: Rng) -> int:
        return _ok(lib().rtw_texture_marble(self._b, scale, rng._p))

    def texture_image_rgb8(self, rgb: np.ndarray) -> int:
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
        h, w, _ = rgb.shape
        return _ok(lib().rtw_texture_image_rgb8(self._b, rgb.ctypes.data_as(C.POINTER(C.c_uint8)), w, h))

    # materials
    def material_lambert(self, albedo: int) -> int:
        return _ok(lib().rtw_material_lambert(self._b, albedo))

    def material_lambert_solid(self, color) -> int:
        return self.material_lambert(self.texture_solid(color))

    def material_metal_solid(self, color, fuzz: float) -> int:
        return _ok(lib().rtw_material_metal(self._b, self.texture_solid(color), fuzz))

    def material_dielectric(self, index_of_refraction: float) -> int:
        return _ok(lib().rtw_material_dielectric(self._b, index_of_refraction))

    def material_diffuse_light_solid(self, color) -> int:
        return _ok(lib().rtw_material_diffuse_light(self._b, self.texture_solid(color)))

    def material_isotropic_solid(self, color) -> int:
        return _ok(lib().rtw_material_isotropic(self._b, self.texture_solid(color)))

    # nodes
    def new_group(self) -> NodeBuilder:
        return NodeBuilder(self, _ok(lib().rtw_node_group(self._b)))

    def new_obj_sphere(self, radius: float, material: int) -> NodeBuilder:
        return NodeBuilder(self, _ok(lib().rtw_node_sphere(self._b, radius, material)))

    def new_obj_sphere_ground(self, radius: float, height: float, material: int) -> NodeBuilder:
        return self.new_obj_sphere(radius, material).translate((0.0, np.float32(height) - np.float32(radius), 0.0))

    def _rect(self, plane: int, position, s0: float, s1: float, material: int) -> NodeBuilder:
        c = (C.c_float * 3)(*position)
        return NodeBuilder(self, _ok(lib().rtw_node_rect(self._b, plane, c, s0, s1, material)))

    def new_obj_rect_yz(self, position, size0, size1, material) -> NodeBuilder:
        return self._rect(N.PLANE_YZ, position, size0, size1, material)

    def new_obj_rect_xz(self, position, size0, size1, material) -> NodeBuilder:
        return self._rect(N.PLANE_XZ, position, size0, size1, material)

    def new_obj_rect_xy(self, position, size0, size1, material) -> NodeBuilder:
        return self._rect(N.PLANE_XY, position, size0, size1, material)

    def new_obj_box(self, width: float, height: float, depth: float, material: int) -> NodeBuilder:
        return NodeBuilder(self, _ok(lib().rtw_node_box(self._b, width, height, depth, material)))

    def new_mesh(self, triangles: np.ndarray, material: int) -> NodeBuilder:
        """new_mesh_from_file_obj_uniform_material with an already-parsed mesh (n x 24 f32)."""
        t = np.ascontiguousarray(triangles, dtype=np.float32).reshape(-1, 24)
        return NodeBuilder(
            self, _ok(lib().rtw_node_mesh(self._b, t.ctypes.data_as(C.POINTER(C.c_float)), len(t), material))
        )

    def new_mesh_from_obj_text(self, text: str, material: int) -> NodeBuilder:
        return self.new_mesh(load_obj_mesh(text), material)


def load_obj_mesh(text: str | bytes) -> np.ndarray:
    """obj_loader.rs:7-22 load_obj_mesh (fan-triangulation quirk kept): (n, 24) f32 records
    [positions(3x3), normals(3x3), uvs(3x2)]."""
    data = text.encode() if isinstance(text, str) else bytes(text)
    out = C.POINTER(C.c_float)()
    n = C.c_int32()
    check(lib().rtw_obj_parse(data, len(data), C.byref(out), C.byref(n)))
    try:
        arr = np.ctypeslib.as_array(out, (max(1, n.value) * 24,))[: n.value * 24].copy()
    finally:
        lib().rtw_free(out)
    return arr.reshape(-1, 24)


@dataclass
class AssetSet:
    suzanne: np.ndarray | None = None
    cube: np.ndarray | None = None
    earth: np.ndarray | None = None  # (H, W, 3) uint8
    _keep: list = field(default_factory=list)

    def raw(self) -> N.Assets:
        a = N.Assets()
        if self.suzanne is not None:
            s = np.ascontiguousarray(self.suzanne, np.float32)
            self._keep.append(s)
            a.suzanne_tris = s.ctypes.data_as(C.POINTER(C.c_float))
            a.suzanne_count = len(s)
        if self.cube is not None:
            c = np.ascontiguousarray(self.cube, np.float32)
            self._keep.append(c)
            a.cube_tris = c.ctypes.data_as(C.POINTER(C.c_float))
            a.cube_count = len(c)
        if self.earth is not None:
            e = np.ascontiguousarray(self.earth, np.uint8)
            self._keep.append(e)
            a.earth_rgb = e.ctypes.data_as(C.POINTER(C.c_uint8))
            a.earth_height, a.earth_width = e.shape[:2]
        return a


DEMO_WORLDS = (
    "final_scene1",
    "final_scene2",
    "cornell_box",
    "cornell_box_smoke",
    "cornell_cube",
    "suzanne",
    "earth_mapped",
    "earth_motion",
    "moving_spheres",
    "perlin_spheres",
    "simple_plane",
    "defocus_blur",
)


def demo_world(name: str, assets: AssetSet | None = None) -> World:
    """create_world_<name> (demo_worlds.rs) with the scene RNG seeded as main.rs:24."""
    if assets is None:
        from .assets import load_assets

        assets = load_assets()
    raw = assets.raw()
    out = C.c_void_p()
    check(lib().rtw_demo_world(name.encode(), C.byref(raw), C.byref(out)))
    return World(out.value)
