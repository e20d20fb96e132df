"""gr_raytracer_amd — MI355X-native hot path of mdreem/gr_raytracer.

The per-pixel RKF45 null-geodesic solve (Schwarzschild, Kerr-Schild, Kerr-BL,
Euclidean), the Sphere/Disc chord intersection and the redshift/beaming shade run in
hand-written HIP kernels for gfx950 (gr_raytracer_amd/csrc/device).  The host side
(TOML scenes, camera tetrads, LUTs, CLI) is C++ behind the C ABI in include/grt_api.h;
this package is a thin ctypes mirror of that surface.
"""
from ._lib import GrtError, lib  # noqa: F401
from .scene import (  # noqa: F401
    BlackBody, Bitmap, Checker, GlobalOpts, HostScene, RenderResult, Scene, SceneBuilder, blackbody_xyz,
    build_camera, cartesian_to_boyer_lindquist, cartesian_to_spherical, default_adaptive, device_count,
    kerr_temperature_lut, load_scene, r_isco, srgb_to_xyza, stationary_velocity, xyz_to_srgb8, Trajectories, ray_at,
    write_trajectory_csv, format_f64, set_arithmetic, get_arithmetic,
)

__all__ = [
    "GrtError", "lib", "BlackBody", "Bitmap", "Checker", "GlobalOpts", "HostScene", "RenderResult", "Scene",
    "SceneBuilder", "blackbody_xyz", "build_camera", "cartesian_to_boyer_lindquist", "cartesian_to_spherical",
    "default_adaptive", "device_count", "kerr_temperature_lut", "load_scene", "r_isco", "srgb_to_xyza",
    "stationary_velocity", "xyz_to_srgb8", "Trajectories", "ray_at", "write_trajectory_csv", "format_f64",
    "set_arithmetic", "get_arithmetic",
]
