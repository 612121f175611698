"""rt_mi355x — MI355X-native drop-in for rust-ray-tracing's per-pixel sample loop.

Python view of the C ABI in include/rt_mi355x.h (the product is the HIP library
lib/librt_mi355x.so; this package only binds it and mirrors the reference's host types).
"""
from . import abi
from .abi import load_library, RtError
from .scene import Camera, Dielectric, FlatScene, Lambertian, Metal, Scene, Sphere, MAIN_CAMERA, camera_new_py
from .renderer import GpuRenderer, RenderStat, Renderer
from . import scenes
from . import parallel
from . import toml_scene
from .toml_scene import Panic, load_scene, scene_from_toml

__all__ = [
    "abi", "load_library", "RtError", "Camera", "Dielectric", "FlatScene", "Lambertian", "Metal", "Scene",
    "Sphere", "MAIN_CAMERA", "camera_new_py", "GpuRenderer", "RenderStat", "Renderer", "scenes", "parallel", "toml_scene", "Panic", "load_scene", "scene_from_toml",
]
