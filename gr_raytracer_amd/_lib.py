"""ctypes binding of include/grt_api.h (the C ABI of libgrt.so).

The structures below mirror the C layout field for field.  Loading fails loudly when
the HIP library has not been built: there is no CPU fallback in the product path.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("GRT_LIB", str(PKG_DIR / "lib" / "libgrt.so")))

GRT_ABI_VERSION = 3
GRT_MAX_OBJECTS = 8
GRT_MAX_HITS = 16

# enums (grt_api.h)
GEOM_EUCLIDEAN, GEOM_SCHWARZSCHILD, GEOM_KERR, GEOM_KERR_BL, GEOM_EUCLIDEAN_SPHERICAL = 0, 1, 2, 3, 4
TEX_BITMAP, TEX_CHECKER, TEX_BLACKBODY = 0, 1, 2
OBJ_SPHERE, OBJ_DISC, OBJ_VOLUMETRIC_DISC = 0, 1, 2
TEMP_CONSTANT, TEMP_KERR_LUT = 0, 1
CLASS_ESCAPED, CLASS_CAPTURED, CLASS_HIT = 0, 1, 2
STATUS_OK, ERR_MAX_STEPS, ERR_NO_CIRCULAR_ORBIT, ERR_BELOW_RISCO, ERR_NON_FINITE_RADIUS = 0, 1, 2, 3, 4
FLAG_HIT_OVERFLOW = 0x80
STOP_NONE, STOP_HORIZON, STOP_CELESTIAL, STOP_NAN, STOP_CLOSED_ORBIT = 0, 1, 2, 3, 4

_d = C.c_double
_pd = C.POINTER(C.c_double)


class TextureDesc(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("_pad", C.c_int32), ("beaming_exponent", _d),
        ("rgba", C.POINTER(C.c_uint8)), ("width", C.c_uint32), ("height", C.c_uint32),
        ("checker_width", _d), ("checker_height", _d), ("c1", _d * 4), ("c2", _d * 4),
    ]


class ObjectDesc(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("temp_kind", C.c_int32), ("radius", _d), ("center", _d * 3),
        ("temperature", _d), ("inner_radius", _d), ("outer_radius", _d),
        ("temp_constant", _d), ("r_isco", _d), ("lut_r", _pd), ("lut_t", _pd),
        ("lut_n", C.c_uint32), ("_pad2", C.c_uint32), ("texture", TextureDesc),
        # VolumetricDisc (volumetric_disc.rs:21-95)
        ("axis", _d * 3), ("thickness", _d), ("march_step_size", _d), ("density_multiplier", _d),
        ("brightness_reference_temperature", _d), ("absorption", _d), ("scattering", _d),
        ("noise_scale", _d * 3), ("noise_offset", _d), ("march_max_steps", C.c_uint64),
        ("num_octaves", C.c_uint32), ("perlin_seed", C.c_uint32),
    ]


class CameraDesc(C.Structure):
    _fields_ = [
        ("position", _d * 4), ("velocity", _d * 4), ("tetrad", (_d * 4) * 4), ("alpha", _d),
        ("tan_half_alpha", _d), ("rows", C.c_int64), ("cols", C.c_int64),
        ("spatial_signature", _d), ("spatial_handedness", _d), ("sin_theta", _d), ("cos_theta", _d),
    ]


class SceneDesc(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32), ("geometry", C.c_int32), ("radius", _d), ("a", _d),
        ("horizon_epsilon", _d), ("max_steps", C.c_uint64), ("max_radius", _d), ("step_size", _d),
        ("epsilon", _d), ("camera", CameraDesc), ("celestial", TextureDesc),
        ("celestial_temperature", _d), ("n_objects", C.c_uint32), ("_pad", C.c_uint32),
        ("objects", ObjectDesc * GRT_MAX_OBJECTS), ("bb_log_t", _pd), ("bb_xyz", _pd),
        ("bb_n", C.c_uint32), ("_pad3", C.c_uint32), ("srgb_to_linear", _d * 256),
        ("object_hit_opacity_threshold", _d),
    ]


class GlobalOpts(C.Structure):
    _fields_ = [
        ("width", C.c_int64), ("height", C.c_int64), ("step_size", _d), ("max_steps", C.c_uint64),
        ("max_radius", _d), ("epsilon", _d), ("camera_position", _d * 3), ("phi", _d),
        ("theta", _d), ("psi", _d), ("tone_mapping", C.c_int32), ("show_sampling_mask", C.c_int32),
        ("sampling_mask_color", C.c_uint8 * 3), ("_pad", C.c_uint8 * 5),
    ]


class AdaptiveConfig(C.Structure):
    _fields_ = [
        ("enabled", C.c_int32), ("samples_per_axis", C.c_uint32),
        ("luminance_contrast_threshold", _d), ("opacity_contrast_threshold", _d),
        ("has_minimum_luminance", C.c_int32), ("exclude_background_contrast", C.c_int32),
        ("minimum_luminance", _d), ("object_hit_opacity_threshold", _d),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("accepted_steps", C.c_uint64), ("attempts", C.c_uint64), ("rays", C.c_uint64),
        ("hit_overflows", C.c_uint64), ("kernel_ms", _d), ("march_jobs", C.c_uint64),
        ("march_samples", C.c_uint64), ("march_noise_samples", C.c_uint64), ("march_emit_samples", C.c_uint64),
    ]


class Offsets(C.Structure):
    _fields_ = [
        ("count", C.c_uint64), ("pixel_index", C.POINTER(C.c_uint32)), ("dx", _pd), ("dy", _pd),
    ]


class AuxOut(C.Structure):
    _fields_ = [("xyza64", _pd), ("steps", C.POINTER(C.c_uint32)), ("stop_reason", C.POINTER(C.c_uint8)),
                ("hits", C.POINTER(C.c_uint32))]


class RowShard(C.Structure):
    _fields_ = [("band_rows", C.c_uint32), ("shard", C.c_uint32), ("n_shards", C.c_uint32)]


class SubsampleFailures(C.Structure):
    _fields_ = [("capacity", C.c_uint64), ("pixel", C.POINTER(C.c_uint32)), ("sample", C.POINTER(C.c_uint32)),
                ("status", C.POINTER(C.c_uint8)), ("count", C.c_uint64), ("stop", C.POINTER(C.c_uint8)),
                ("steps", C.POINTER(C.c_uint32))]


GRT_MULTI_MAX_DEVICES = 16


class FrameOut(C.Structure):
    """grt_frame_out: host outputs of grt_render_frame_multi, frame order (NULL: not gathered)."""
    _fields_ = [("xyza", C.POINTER(C.c_float)), ("xyza64", _pd), ("ray_class", C.POINTER(C.c_uint8)),
                ("status", C.POINTER(C.c_uint8)), ("stop", C.POINTER(C.c_uint8)), ("steps", C.POINTER(C.c_uint32))]


class MultiReport(C.Structure):
    _fields_ = [("n_devices", C.c_uint32), ("record_bytes", C.c_uint32), ("attempts", C.c_uint32),
                ("_pad", C.c_uint32), ("wall_ms", _d), ("gather_ms", _d), ("allgather_ms", _d),
                ("trace_ms", _d * GRT_MULTI_MAX_DEVICES), ("accepted_steps", C.c_uint64 * GRT_MULTI_MAX_DEVICES),
                ("rows", C.c_uint64 * GRT_MULTI_MAX_DEVICES)]


class Health(C.Structure):
    _fields_ = [
        ("rays", C.c_uint64), ("failed", C.c_uint64), ("null_violations", C.c_uint64), ("max_null", _d),
        ("kk_drift_rays", C.c_uint64), ("max_kk_drift", _d), ("n_constants", C.c_uint32), ("_pad", C.c_uint32),
        ("constant_drift_rays", C.c_uint64 * 3), ("max_constant_drift", _d * 3),
    ]


class GrtError(RuntimeError):
    pass


_lib = None


def lib() -> C.CDLL:
    """The loaded libgrt.so.  Raises if the HIP library is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise GrtError(
            f"{LIB_PATH} not found: the HIP extension is not built "
            "(run `python -c 'import __graft_entry__; __graft_entry__.build()'` or "
            "`make -C gr_raytracer_amd/csrc`). There is no CPU fallback.")
    # libgrt.so and torch's ROCm build both need libamdhip64.so.7; the first one loaded
    # serves the whole process.  torch refuses a HIP runtime other than its own ("No HIP
    # GPUs are available"), while libgrt runs on either, so torch (plumbing for device
    # buffers, streams and torch.distributed) is loaded first when it is installed.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(str(LIB_PATH))
    vp, u32, u64, i32, i64 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32, C.c_int64
    sigs = {
        "grt_last_error": (C.c_char_p, []),
        "grt_device_count": (C.c_int, []),
        "grt_source_hash": (C.c_char_p, []),
        "grt_default_global_opts": (None, [C.POINTER(GlobalOpts)]),
        "grt_default_adaptive_config": (None, [C.POINTER(AdaptiveConfig)]),
        "grt_host_scene_load": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(GlobalOpts), C.POINTER(vp)]),
        "grt_host_scene_desc": (C.POINTER(SceneDesc), [vp]),
        "grt_host_scene_log": (C.c_char_p, [vp]),
        "grt_host_geometry_load": (C.c_int, [C.c_char_p, C.POINTER(GlobalOpts), C.POINTER(vp)]),
        "grt_host_scene_adaptive": (None, [vp, C.POINTER(AdaptiveConfig)]),
        "grt_host_scene_destroy": (C.c_int, [vp]),
        "grt_camera_build": (C.c_int, [i32, _d, _d, _pd, _pd, _d, i64, i64, _d, _d, _d, C.POINTER(CameraDesc)]),
        "grt_stationary_velocity": (C.c_int, [i32, _d, _d, _pd, _pd]),
        "grt_zamo_velocity": (C.c_int, [i32, _d, _d, _pd, _pd]),
        "grt_cartesian_to_spherical": (None, [_pd, _pd]),
        "grt_cartesian_to_boyer_lindquist": (None, [_d, _pd, _pd]),
        "grt_kerr_temperature_lut": (C.c_int, [_d, _d, _d, _d, u32, _pd, _pd, _pd]),
        "grt_r_isco": (_d, [_d, _d]),
        "grt_blackbody_lut": (C.c_int, [u32, _pd, _pd]),
        "grt_blackbody_xyz": (None, [_d, _d, _pd]),
        "grt_srgb_to_xyza": (None, [C.c_uint8, C.c_uint8, C.c_uint8, C.c_uint8, _pd]),
        "grt_perlin_permutation": (None, [u32, C.POINTER(C.c_uint8)]),
        "grt_volumetric_frame": (None, [_pd, _pd, _pd, _pd]),
        "grt_xyz_to_srgb8": (C.c_int, [_pd, C.c_size_t, i32, _d, C.POINTER(C.c_uint8)]),
        "grt_linear_max": (None, [_pd, C.c_size_t, _d, _pd]),
        "grt_xyz_to_srgb": (None, [_pd, _d, C.POINTER(C.c_uint8)]),
        "grt_blackbody_spectrum": (C.c_int, [_d, _d, _d, _d, u32, u32, i32, C.POINTER(C.c_uint8)]),
        "grt_tonemap": (C.c_int, [_pd, C.c_size_t, i32, _d, _pd, C.POINTER(C.c_uint8)]),
        "grt_scene_create": (C.c_int, [C.POINTER(SceneDesc), C.POINTER(vp)]),
        "grt_scene_destroy": (C.c_int, [vp]),
        "grt_render_pixels": (C.c_int, [vp, C.c_int, u32, u32, u32, u32, C.POINTER(Offsets),
                                        C.POINTER(C.c_float), C.POINTER(C.c_uint8), C.POINTER(C.c_uint8),
                                        C.POINTER(AuxOut), C.POINTER(Stats)]),
        "grt_render_pixels_async": (C.c_int, [vp, C.c_int, vp, u32, u32, u32, u32, vp, vp, vp, vp, vp, vp, vp]),
        "grt_render_section": (C.c_int, [vp, C.c_int, u32, u32, u32, u32, C.POINTER(AdaptiveConfig), _pd, _pd,
                                         C.POINTER(C.c_uint8), C.POINTER(C.c_uint64), C.POINTER(Stats),
                                         C.POINTER(C.c_uint8)]),
        "grt_set_launch_config": (C.c_int, [C.c_int, C.c_int]),
        "grt_set_schedule": (C.c_int, [C.c_int]),
        "grt_set_two_ended": (C.c_int, [C.c_int]),
        "grt_set_tail": (C.c_int, [C.c_longlong]),
        "grt_health_pixels": (C.c_int, [C.c_void_p, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                        C.POINTER(Health), _pd]),
        "grt_tail_handoffs": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_uint64)]),
        "grt_tail_report": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_double),
                                      C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_uint64]),
        "grt_shard_row_count": (u32, [u32, C.POINTER(RowShard)]),
        "grt_shard_frame_row": (u32, [u32, C.POINTER(RowShard)]),
        "grt_render_shard": (C.c_int, [vp, C.c_int, C.POINTER(RowShard), C.POINTER(C.c_float), C.POINTER(C.c_uint8),
                                       C.POINTER(C.c_uint8), C.POINTER(AuxOut), C.POINTER(Stats)]),
        "grt_render_shard_async": (C.c_int, [vp, C.c_int, vp, C.POINTER(RowShard), vp, vp, vp, vp, vp, vp, vp]),
        "grt_hit_pool_reserve": (C.c_int, [vp, C.c_int, u64, C.POINTER(C.c_uint64)]),
        "grt_set_hit_pool_min": (C.c_int, [u64]),
        "grt_set_sub_chunk": (C.c_int, [u64]),
        "grt_adaptive_min_luminance": (_d, [_pd, u64, C.POINTER(AdaptiveConfig)]),
        "grt_adaptive_min_luminance_device": (C.c_int, [C.c_int, vp, vp, u32, u64, C.POINTER(AdaptiveConfig),
                                                        C.POINTER(_d)]),
        "grt_supersample_shard": (C.c_int, [vp, C.c_int, vp, C.POINTER(RowShard), C.POINTER(AdaptiveConfig), _d, vp, vp,
                                            _pd, vp, C.POINTER(C.c_uint64), vp]),
        "grt_supersample_shard_device": (C.c_int, [vp, C.c_int, vp, C.POINTER(RowShard), C.POINTER(AdaptiveConfig), _d,
                                                   vp, vp, vp, _pd, vp, vp, vp, C.POINTER(SubsampleFailures)]),
        "grt_adaptive_floor_device": (C.c_int, [vp, C.c_int, vp, vp, u32, u64, vp]),
        "grt_render_section_ex": (C.c_int, [vp, C.c_int, u32, u32, u32, u32, C.POINTER(AdaptiveConfig), _pd, _pd,
                                            C.POINTER(C.c_uint8), C.POINTER(C.c_uint64), C.POINTER(Stats),
                                            C.POINTER(C.c_uint8), C.POINTER(SubsampleFailures),
                                            C.POINTER(C.c_uint8), C.POINTER(C.c_uint32)]),
        "grt_write_png_rgb": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint8), u32, u32]),
        "grt_write_hdr_xyz": (C.c_int, [C.c_char_p, _pd, u32, u32]),
        "grt_linear_max_async": (C.c_int, [C.c_int, vp, vp, u64, _d, vp]),
        "grt_tonemap_async": (C.c_int, [C.c_int, vp, vp, u64, i32, _d, vp, vp]),
        "grt_xyz_to_srgb8_device": (C.c_int, [C.c_int, _pd, C.c_size_t, i32, _d, C.POINTER(C.c_uint8)]),
        "grt_trace_pixels": (C.c_int, [vp, C.c_int, u64, _pd, _pd, u64, _pd, C.POINTER(C.c_uint64),
                                       C.POINTER(C.c_uint8), C.POINTER(C.c_uint8)]),
        "grt_trace_rays": (C.c_int, [vp, C.c_int, u64, _pd, _pd, u64, _pd, C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_uint8), C.POINTER(C.c_uint8)]),
        "grt_ray_at": (C.c_int, [i32, _d, _d, _pd, _pd, _pd, _pd]),
        "grt_write_trajectory_csv": (C.c_int, [C.c_char_p, i32, _d, _pd, u64]),
        "grt_format_f64": (C.c_size_t, [_d, C.c_char_p, C.c_size_t]),
        "grt_render_frame_multi": (C.c_int, [vp, C.c_int, C.POINTER(C.c_int), u32, C.POINTER(AdaptiveConfig), _pd,
                                             C.POINTER(FrameOut), C.POINTER(C.c_uint64), C.POINTER(Stats),
                                             C.POINTER(SubsampleFailures), C.POINTER(MultiReport)]),
        "grt_multi_release": (None, []),
        "grt_set_arithmetic": (C.c_int, [C.c_int]),
        "grt_get_arithmetic": (C.c_int, []),
    }
    # GRT_LIB_ALLOW_MISSING=1 (tools/time_variants.py only) binds an older experimental
    # build that lacks newer entry points; by default a missing symbol is an error.
    # It also skips the source stamp check below (such a build is not the checkout's).
    allow_missing = os.environ.get("GRT_LIB_ALLOW_MISSING") == "1"
    for name, (res, args) in sigs.items():
        if allow_missing and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if not allow_missing:
        check_source_stamp(L)
    _lib = L
    return L


def check_source_stamp(L) -> str:
    """The library's grt_source_hash() must equal the checkout's source hash
    (source_hash.py): a prebuilt libgrt.so from other sources is refused."""
    from .source_hash import source_hash

    stamp = L.grt_source_hash().decode()
    want = source_hash()
    if stamp != want:
        raise GrtError(f"{LIB_PATH} was built from other sources (stamp {stamp[:16]}, checkout {want[:16]}): "
                       "rebuild it (make -C gr_raytracer_amd/csrc)")
    return stamp


def source_stamp() -> str:
    """The loaded library's source hash (bench.py and smoke() print it)."""
    return lib().grt_source_hash().decode()


EXPORTED_SYMBOLS = [
    "grt_last_error", "grt_device_count", "grt_source_hash", "grt_default_global_opts", "grt_default_adaptive_config",
    "grt_host_scene_load", "grt_host_geometry_load", "grt_host_scene_desc", "grt_host_scene_log", "grt_host_scene_adaptive", "grt_host_scene_destroy",
    "grt_camera_build", "grt_stationary_velocity", "grt_zamo_velocity", "grt_cartesian_to_spherical",
    "grt_cartesian_to_boyer_lindquist", "grt_kerr_temperature_lut", "grt_r_isco", "grt_blackbody_lut",
    "grt_blackbody_xyz", "grt_srgb_to_xyza", "grt_perlin_permutation", "grt_volumetric_frame", "grt_xyz_to_srgb8", "grt_xyz_to_srgb", "grt_blackbody_spectrum", "grt_linear_max", "grt_tonemap", "grt_scene_create", "grt_scene_destroy",
    "grt_render_pixels", "grt_render_pixels_async", "grt_render_section", "grt_set_launch_config", "grt_set_schedule", "grt_set_two_ended", "grt_set_tail", "grt_tail_handoffs", "grt_health_pixels", "grt_tail_report",
    "grt_shard_row_count", "grt_shard_frame_row", "grt_render_shard", "grt_render_shard_async", "grt_hit_pool_reserve", "grt_set_hit_pool_min", "grt_set_sub_chunk",
    "grt_linear_max_async", "grt_tonemap_async", "grt_xyz_to_srgb8_device", "grt_trace_pixels", "grt_trace_rays",
    "grt_ray_at", "grt_write_trajectory_csv", "grt_format_f64", "grt_adaptive_min_luminance", "grt_adaptive_min_luminance_device", "grt_supersample_shard",
    "grt_supersample_shard_device", "grt_adaptive_floor_device", "grt_render_section_ex",
    "grt_write_png_rgb", "grt_write_hdr_xyz", "grt_render_frame_multi", "grt_multi_release",
    "grt_set_arithmetic", "grt_get_arithmetic",
]


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().grt_last_error().decode(errors="replace")
        raise GrtError(f"{what} failed ({rc}): {msg}")


def dptr(arr) -> _pd:
    return arr.ctypes.data_as(_pd)


def ptr(arr, ctype):
    return arr.ctypes.data_as(C.POINTER(ctype))


def device_code_sha256(path: Path = LIB_PATH) -> str:
    """SHA-256 of the gfx950 device code inside libgrt.so (its ELF `.hip_fatbin`
    section: every kernel's code object).  PMC summaries under profiles/ record it, and
    bench.py refuses a summary taken from another build."""
    import hashlib
    import struct

    data = Path(path).read_bytes()
    if data[:4] != b"\x7fELF" or data[4] != 2:
        raise GrtError(f"{path}: not an ELF64 file")
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def section(i):
        name, _type, _flags, _addr, off, size = struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)
        return name, off, size

    _, str_off, _ = section(shstrndx)
    for i in range(shnum):
        name, off, size = section(i)
        end = data.index(b"\0", str_off + name)
        if data[str_off + name:end] == b".hip_fatbin":
            return hashlib.sha256(data[off:off + size]).hexdigest()
    raise GrtError(f"{path}: no .hip_fatbin section")


def _elf_sections(data: bytes, base: int = 0):
    """{name: (offset, size, link, entsize)} of an ELF64 image starting at data[base:]."""
    import struct

    shoff, = struct.unpack_from("<Q", data, base + 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, base + 0x3A)
    raw = [struct.unpack_from("<IIQQQQIIQQ", data, base + shoff + i * shentsize) for i in range(shnum)]
    str_off = base + raw[shstrndx][4]
    out = {}
    for name, _t, _f, _a, off, size, link, _info, _al, entsize in raw:
        nm = data[str_off + name:data.index(b"\0", str_off + name)].decode()
        out[nm] = (base + off, size, raw[link][4] + base if link < len(raw) else 0, entsize)
    return out


def _mask_pc_relative(code: bytearray) -> None:
    """Zero the link-time displacements of `s_getpc_b64; s_add_u32 lit; s_addc_u32 lit`
    (the address of a global table: they move when other kernels change size)."""
    import struct

    for i in range(0, len(code) - 20, 4):
        w0, w1, _, w3 = struct.unpack_from("<IIII", code, i)
        if (w0 & 0xFF80FF00) == 0xBE801C00 and (w1 >> 24) == 0x80 and ((w1 >> 8) & 0xFF) == 0xFF \
                and (w3 >> 24) == 0x82 and ((w3 >> 8) & 0xFF) == 0xFF:
            code[i + 8:i + 12] = bytes(4)
            code[i + 16:i + 20] = bytes(4)


def _gfx950_code_objects(data: bytes, path) -> list:
    """Offsets of the gfx950 code objects in the `.hip_fatbin` section: one offload bundle
    per translation unit with device code, back to back."""
    import struct

    fb_off, fb_size, _, _ = _elf_sections(data)[".hip_fatbin"]
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    if data[fb_off:fb_off + len(magic)] != magic:
        raise GrtError(f"{path}: .hip_fatbin is not an uncompressed offload bundle")
    out = []
    b = fb_off
    while b >= 0 and b < fb_off + fb_size:
        p = b + len(magic)
        n, = struct.unpack_from("<Q", data, p)
        p += 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            if "gfx950" in data[p + 24:p + 24 + tlen].decode():
                out.append(b + off)
            p += 24 + tlen
        b = data.find(magic, p, fb_off + fb_size)
    if not out:
        raise GrtError(f"{path}: no gfx950 code object in the bundle")
    return out


def kernel_code_sha256(symbol: str, path: Path = LIB_PATH) -> str:
    """SHA-256 of ONE kernel's gfx950 machine code and kernel descriptor inside
    libgrt.so: the bytes of the function symbol `symbol` (mangled name) and of
    `symbol.kd` in the gfx950 code object of the `.hip_fatbin` offload bundle.  A PMC
    summary records it for the kernel it measured, so adding or changing an unrelated
    kernel does not invalidate it (a change of this kernel's code, register counts or
    LDS size does)."""
    import hashlib
    import struct

    data = Path(path).read_bytes()
    co = None
    for c in _gfx950_code_objects(data, path):  # the code object that defines the kernel
        sym_off, sym_size, str_off, entsize = _elf_sections(data, c)[".symtab"]
        names = {data[str_off + struct.unpack_from("<I", data, sym_off + k * entsize)[0]:
                      data.index(b"\0", str_off + struct.unpack_from("<I", data, sym_off + k * entsize)[0])].decode()
                 for k in range(sym_size // entsize)}
        if symbol in names:
            co = c
            break
    if co is None:
        raise GrtError(f"{path}: kernel symbol {symbol} not found")
    secs = _elf_sections(data, co)
    sym_off, sym_size, str_off, entsize = secs[".symtab"]
    h = hashlib.sha256()
    found = 0
    for want in (symbol, symbol + ".kd"):
        for k in range(sym_size // entsize):
            st_name, st_info, _o, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", data, sym_off + k * entsize)
            nm = data[str_off + st_name:data.index(b"\0", str_off + st_name)].decode()
            if nm != want:
                continue
            # locate the symbol's bytes through its section's address/offset
            shoff, = struct.unpack_from("<Q", data, co + 0x28)
            shentsize, = struct.unpack_from("<H", data, co + 0x3A)
            _n, _t, _f, s_addr, s_off, _s, _l, _i, _al, _e = struct.unpack_from("<IIQQQQIIQQ", data,
                                                                                  co + shoff + st_shndx * shentsize)
            start = co + s_off + (st_value - s_addr)
            body = bytearray(data[start:start + st_size])
            if want.endswith(".kd"):
                body[16:24] = bytes(8)  # kernel_code_entry_byte_offset: where the linker placed the code
            else:
                _mask_pc_relative(body)
            h.update(want.encode() + b"\0" + bytes(body))
            found += 1
            break
    if found != 2:
        raise GrtError(f"{path}: kernel symbol {symbol} (and its .kd) not found")
    return h.hexdigest()


def kernel_symbols(path: Path = LIB_PATH) -> list:
    """Mangled names of the kernels in libgrt.so's gfx950 code objects (every unit)."""
    import struct

    data = Path(path).read_bytes()
    out = []
    for co in _gfx950_code_objects(data, path):
        sym_off, sym_size, str_off, entsize = _elf_sections(data, co)[".symtab"]
        for k in range(sym_size // entsize):
            st_name, = struct.unpack_from("<I", data, sym_off + k * entsize)
            nm = data[str_off + st_name:data.index(b"\0", str_off + st_name)].decode()
            if nm.endswith(".kd"):
                out.append(nm[:-3])
    return out


def kernel_symbol(demangled: str, path: Path = LIB_PATH) -> str:
    """Mangled name of a `grt::name<int-or-bool, ...>` (or `grt::ns::name<...>`) kernel,
    e.g. "grt::integrate_kernel<1, false>" -> "_ZN3grt16integrate_kernelILi1ELb0EE..."."""
    import re

    m = re.fullmatch(r"grt::(?:(\w+)::)?(\w+)<([^>]*)>", demangled.strip())
    if not m:
        raise GrtError(f"cannot mangle {demangled!r}")
    ns, name, args = m.group(1), m.group(2), [a.strip() for a in m.group(3).split(",")]
    enc = "".join("Lb1E" if a == "true" else "Lb0E" if a == "false" else f"Li{int(a)}E" for a in args)
    prefix = f"_ZN3grt{len(ns)}{ns}{len(name)}{name}I{enc}E" if ns else f"_ZN3grt{len(name)}{name}I{enc}E"
    hits = [k for k in kernel_symbols(path) if k.startswith(prefix)]
    if len(hits) != 1:
        raise GrtError(f"{demangled}: {len(hits)} matching kernel symbols")
    return hits[0]
