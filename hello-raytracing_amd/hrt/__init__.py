"""hrt — MI355X-native path tracer (drop-in for hucancode/hello-raytracing's per-pixel ray loop).

The compute path is lib/libhrt.so (HIP kernels for gfx950 behind the C-ABI of include/hrt.h); this
package is the host-side mirror of the reference's Rust scene API plus ctypes plumbing.
"""
from ._lib import (LIB_PATH, RT_FOLD_AUTO, RT_FOLD_BUFFER, RT_FOLD_NEXT, RT_FOLD_RING, RT_MODE_MIXED, RT_SCHEDULE_AUTO, RT_SCHEDULE_QUEUE, RT_SCHEDULE_TILES, RT_MODE_SPHERE, RT_MODE_TRIS, RtError, RtParams, RtStats,
                   lib)
from .scene import (CAMERA_DTYPE, DIELECTRIC, LAMBERTIAN, MATERIAL_DTYPE, MAX_OBJECT_IN_SCENE, METAL,
                    NODE_DTYPE, PI, SPHERE_DTYPE, TRIANGLE_DTYPE, Camera, ComparisonError, Material, Mesh, OrbitCamera,
                    Renderer, SceneSphere, SceneTris, Sphere, Tree, Vec3, compare_ppm_images, f32,
                    ppm_from_image, read_asset, render_ppm, spheres_array)


def device_count() -> int:
    """Visible HIP devices (0 on a CPU-only host). Does not create a context on the host side."""
    return int(lib().rt_device_count())


__all__ = [
    "LIB_PATH", "RT_FOLD_AUTO", "RT_FOLD_BUFFER", "RT_FOLD_NEXT", "RT_FOLD_RING", "RT_MODE_MIXED", "RT_SCHEDULE_AUTO", "RT_SCHEDULE_QUEUE", "RT_SCHEDULE_TILES", "RT_MODE_SPHERE", "RT_MODE_TRIS", "RtError", "RtParams", "RtStats", "lib",
    "CAMERA_DTYPE", "DIELECTRIC", "LAMBERTIAN", "MATERIAL_DTYPE", "MAX_OBJECT_IN_SCENE", "METAL", "NODE_DTYPE",
    "PI", "SPHERE_DTYPE", "TRIANGLE_DTYPE", "Camera", "ComparisonError", "Material", "Mesh", "OrbitCamera", "Renderer",
    "SceneSphere", "SceneTris", "Sphere", "Tree", "Vec3", "compare_ppm_images", "f32", "ppm_from_image",
    "read_asset", "render_ppm", "spheres_array", "device_count",
]
