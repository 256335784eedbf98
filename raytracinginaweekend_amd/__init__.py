"""raytracinginaweekend_amd: MI355X-native replacement of the per-pixel render loop of
martingleich/RayTracingInAWeekend (src/lib/rendering.rs).

The product is librtw.so (HIP megakernel for gfx950 + host scene builder, C ABI in
include/rtw.h).  This package is its Python face, mirroring the reference's interface:
Camera.build()..., WorldBuilder / NodeBuilder, demo worlds, rendering.render(...).
"""
from . import image_io
from .rendering import (
    DeviceWorld,
    MultiDeviceWorld,
    RenderMode,
    Size2i,
    device_count,
    render,
    render_devices,
    render_params,
)
from .world import (
    DEMO_WORLDS,
    AssetSet,
    BackgroundColor,
    Camera,
    NodeBuilder,
    NodeRef,
    Rng,
    World,
    WorldBuilder,
    demo_world,
    load_obj_mesh,
)

__all__ = [
    "AssetSet",
    "BackgroundColor",
    "Camera",
    "DEMO_WORLDS",
    "DeviceWorld",
    "MultiDeviceWorld",
    "NodeBuilder",
    "NodeRef",
    "RenderMode",
    "Rng",
    "Size2i",
    "World",
    "WorldBuilder",
    "demo_world",
    "device_count",
    "load_obj_mesh",
    "render",
    "render_devices",
    "render_params",
]
