"""ctypes wrapper of the oracle (oracle/grt_oracle.cpp).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg to check / time the reference algorithm on the CPU.  The product
(gr_raytracer_amd) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SO = HERE / "_build" / "liboracle.so"
_lib = None

_d, _pd = C.c_double, C.POINTER(C.c_double)
_u8p, _u32p, _u64p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return SO


def lib():
    global _lib
    if _lib is None:
        if not SO.exists():
            build()
        L = C.CDLL(str(SO))
        vp = C.c_void_p
        L.oracle_color_of_ray.argtypes = [vp, C.c_int64, C.c_int64, C.c_int, _d, _d, _pd, _u8p, _u8p, _u8p, _u64p, _u64p]
        L.oracle_render_pixels.restype = _d
        L.oracle_render_pixels.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, _u32p,
                                           _pd, _pd, _u32p, C.c_uint32, _pd, _u8p, _u8p, _u8p, _u32p, C.c_int,
                                           _u64p, _u64p, _u32p]
        L.oracle_health_pixels.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, _pd, _u8p]
        L.oracle_render_section.restype = C.c_uint64
        L.oracle_render_section.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp, _pd, _pd, _u8p,
                                            C.c_int]
        L.oracle_select_pixels.restype = _d
        L.oracle_select_pixels.argtypes = [_pd, _u8p, C.c_uint32, C.c_uint32, vp, _u8p]
        L.oracle_camera_setup.argtypes = [C.c_int32, _d, _d, _pd, C.c_int, _pd, _d, C.c_int64, C.c_int64, _d, _d, _d,
                                          vp]
        L.oracle_kerr_temperature_lut.argtypes = [_d, _d, _d, _d, C.c_uint32, _pd, _pd, _pd]
        L.oracle_r_isco.restype = _d
        L.oracle_r_isco.argtypes = [_d, _d]
        L.oracle_blackbody_lut.argtypes = [C.c_uint32, _pd, _pd]
        L.oracle_blackbody_xyz.argtypes = [_d, _d, _pd]
        L.oracle_rk_analytic.argtypes = [_d, _pd, _pd]
        L.oracle_integrate_ray.restype = C.c_int64
        L.oracle_integrate_ray.argtypes = [vp, _pd, _pd, _pd, C.c_int64, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.oracle_camera_ray.argtypes = [vp, _d, _d, C.c_int, _d, _d, _pd]
        L.oracle_camera_direction.argtypes = [vp, _d, _d, _pd]
        L.oracle_inner_product.restype = _d
        L.oracle_inner_product.argtypes = [vp, _pd, _pd, _pd]
        L.oracle_stratified_offset.argtypes = [C.c_int64, C.c_int64, C.c_uint64, C.c_uint64, C.c_uint64, _pd, _pd]
        L.oracle_blend.argtypes = [_pd, _pd, _pd]
        L.oracle_texture_color.argtypes = [vp, C.c_int, _d, _d, _d, _d, _pd]
        L.oracle_killing_coefficients.argtypes = [_d, _d, _d, _pd, _pd]
        L.oracle_object_intersects.argtypes = [vp, C.c_int, _pd, _pd, _pd, _pd]
        L.oracle_xyz_to_srgb8.argtypes = [_pd, C.c_uint64, C.c_int, _d, _u8p]
        L.oracle_perlin_table.argtypes = [C.c_uint32, _u8p]
        L.oracle_perlin.restype = _d
        L.oracle_perlin.argtypes = [C.c_uint32, _d, _d, _d]
        L.oracle_should_stop.argtypes = [vp, _pd, C.c_uint64]
        L.oracle_inside_horizon.argtypes = [vp, _pd]
        L.oracle_radial_coordinate.restype = _d
        L.oracle_radial_coordinate.argtypes = [vp, _pd, C.c_int]
        L.oracle_to_cartesian.argtypes = [vp, _pd, _pd]
        L.oracle_stationary_velocity.argtypes = [vp, _pd, _pd]
        L.oracle_circular_orbit_velocity.argtypes = [vp, _pd, _pd]
        L.oracle_geodesic_rhs.argtypes = [vp, _pd, _pd, _pd, _pd, _pd, _pd]
        L.oracle_ks_metric.argtypes = [_d, _d, _d, _d, _d, C.c_int, _pd]
        L.oracle_bl_metric.argtypes = [_d, _d, _d, _d, _pd]
        L.oracle_redshift_static.restype = _d
        L.oracle_redshift_static.argtypes = [vp, _pd, _pd, _d]
        L.oracle_kerr_bl_rhs.argtypes = [_d, _d, _d, _d, _d, _pd, _pd]
        L.oracle_should_supersample_pair.argtypes = [_pd, C.c_int, _pd, C.c_int, vp, _d]
        L.oracle_vdisc_density.restype = _d
        L.oracle_vdisc_density.argtypes = [vp, C.c_int, _pd]
        L.oracle_vdisc_raymarch.argtypes = [vp, C.c_int, _pd, _pd, _pd, C.c_int, _pd, _u64p]
        _lib = L
    return _lib


def _addr(desc):
    return C.cast(C.pointer(desc), C.c_void_p) if not isinstance(desc, C.c_void_p) else desc


def _dp(a):
    return a.ctypes.data_as(_pd)


def color_of_ray(desc, row, col, offset=None):
    xyza = np.zeros(4)
    cls, status, stop = C.c_uint8(), C.c_uint8(), C.c_uint8()
    steps, att = C.c_uint64(), C.c_uint64()
    use, dx, dy = (0, 0.0, 0.0) if offset is None else (1, offset[0], offset[1])
    lib().oracle_color_of_ray(_addr(desc), row, col, use, dx, dy, _dp(xyza), C.byref(cls), C.byref(status),
                              C.byref(stop), C.byref(steps), C.byref(att))
    return {"xyza": xyza, "ray_class": cls.value, "status": status.value, "stop": stop.value,
            "steps": steps.value, "attempts": att.value}


def render_pixels(desc, row0, col0, rows, cols, threads=8, offsets=None, row_list=None):
    """Returns dict with xyza (n,4) f64, ray_class, status, stop, steps, hits (windows with an
    intersection), wall_s, accepted, attempts."""
    if offsets is not None:
        pix = np.ascontiguousarray(offsets[0], np.uint32)
        dx = np.ascontiguousarray(offsets[1], np.float64)
        dy = np.ascontiguousarray(offsets[2], np.float64)
        n = len(pix)
        args = (n, pix.ctypes.data_as(_u32p), _dp(dx), _dp(dy))
    else:
        n = rows * cols if row_list is None else len(row_list) * cols
        args = (0, None, None, None)
    rl = None if row_list is None else np.ascontiguousarray(row_list, np.uint32)
    xyza = np.zeros((n, 4))
    cls, st, stop = np.zeros(n, np.uint8), np.zeros(n, np.uint8), np.zeros(n, np.uint8)
    steps = np.zeros(n, np.uint32)
    hits = np.zeros(n, np.uint32)
    acc, att = C.c_uint64(), C.c_uint64()
    wall = lib().oracle_render_pixels(_addr(desc), row0, col0, rows, cols, *args,
                                      rl.ctypes.data_as(_u32p) if rl is not None else None,
                                      0 if rl is None else len(rl), _dp(xyza), cls.ctypes.data_as(_u8p),
                                      st.ctypes.data_as(_u8p), stop.ctypes.data_as(_u8p), steps.ctypes.data_as(_u32p),
                                      threads, C.byref(acc), C.byref(att), hits.ctypes.data_as(_u32p))
    return {"xyza": xyza, "ray_class": cls, "status": st, "stop": stop, "steps": steps, "hits": hits, "wall_s": wall,
            "accepted": acc.value, "attempts": att.value}


def health_pixels(desc, row0, col0, rows, cols, threads=8):
    """Per-ray invariant monitors (scene.rs:116-124, integrator.rs:91-146): (n, 5) array of
    |k.k| at the camera, largest |k.k| along the path, largest drift of E, L_z, Q; status."""
    n = rows * cols
    out = np.zeros((n, 5))
    st = np.zeros(n, np.uint8)
    lib().oracle_health_pixels(_addr(desc), row0, col0, rows, cols, threads, _dp(out), st.ctypes.data_as(_u8p))
    return out, st


def render_section(desc, from_row, from_col, to_row, to_col, adaptive, mask=None, threads=8):
    n = (to_row - from_row) * (to_col - from_col)
    out = np.zeros((n, 4))
    cls = np.zeros(n, np.uint8)
    m = None if mask is None else np.ascontiguousarray(mask, np.float64)
    nsel = lib().oracle_render_section(_addr(desc), from_row, from_col, to_row, to_col,
                                       C.cast(C.pointer(adaptive), C.c_void_p), _dp(m) if m is not None else None,
                                       _dp(out), cls.ctypes.data_as(_u8p), threads)
    return out, cls, int(nsel)


def select_pixels(xyza, cls, w, h, adaptive):
    """collect_pixels_to_supersample (raytracer.rs:386-458) + the luminance floor (:118-129)
    applied to a given 1-spp section buffer: (bool flags (h*w,), min_luminance)."""
    x = np.ascontiguousarray(xyza, np.float64).reshape(-1, 4)
    c = np.ascontiguousarray(cls, np.uint8)
    assert len(x) == len(c) == w * h
    flags = np.zeros(w * h, np.uint8)
    min_lum = lib().oracle_select_pixels(_dp(x), c.ctypes.data_as(_u8p), w, h,
                                         C.cast(C.pointer(adaptive), C.c_void_p), flags.ctypes.data_as(_u8p))
    return flags.astype(bool), float(min_lum)


# ---- host setup, restated (oracle/host_setup.inc) ----
def camera_setup(camera_desc_type, geometry, radius, a, cart, velocity_mode=0, explicit=None, alpha=np.pi / 4,
                 rows=500, cols=500, phi=0.0, theta=0.0, psi=0.0):
    """Camera::new after the CLI's placement (main.rs:92-104, cli/<geometry>.rs,
    cli/shared.rs:48-77): returns (rc, grt_camera_desc).  velocity_mode 0 static, 1 ZAMO,
    2 explicit."""
    out = camera_desc_type()
    c = np.ascontiguousarray(cart, np.float64)
    e = None if explicit is None else np.ascontiguousarray(explicit, np.float64)
    rc = lib().oracle_camera_setup(geometry, radius, a, _dp(c), velocity_mode, _dp(e) if e is not None else None,
                                   alpha, rows, cols, phi, theta, psi, C.cast(C.pointer(out), C.c_void_p))
    return rc, out


def kerr_temperature_lut(temperature, outer_radius, a, radius, n=1000):
    r, t, ri = np.zeros(n), np.zeros(n), C.c_double()
    rc = lib().oracle_kerr_temperature_lut(temperature, outer_radius, a, radius, n, _dp(r), _dp(t), C.byref(ri))
    return rc, r, t, ri.value


def r_isco(radius, a):
    return lib().oracle_r_isco(radius, a)


def blackbody_lut(n=1000):
    lt, xyz = np.zeros(n), np.zeros((n, 3))
    rc = lib().oracle_blackbody_lut(n, _dp(lt), _dp(xyz))
    assert rc == 0
    return lt, xyz


def blackbody_xyz(temperature, redshift=1.0):
    out = np.zeros(3)
    lib().oracle_blackbody_xyz(temperature, redshift, _dp(out))
    return out


def rk_analytic(t_end):
    y, t = np.zeros(2), C.c_double()
    lib().oracle_rk_analytic(t_end, _dp(y), C.byref(t))
    return y, t.value


def integrate_ray(desc, position, momentum, max_out=200000):
    pos, mom = np.ascontiguousarray(position, np.float64), np.ascontiguousarray(momentum, np.float64)
    out = np.zeros((max_out, 9))
    stop, status = C.c_int32(), C.c_int32()
    n = lib().oracle_integrate_ray(_addr(desc), _dp(pos), _dp(mom), _dp(out), max_out, C.byref(stop), C.byref(status))
    return out[: min(n, max_out)], stop.value, status.value


def camera_ray(desc, row, col, offset=None):
    m = np.zeros(4)
    use, dx, dy = (0, 0.0, 0.0) if offset is None else (1, offset[0], offset[1])
    lib().oracle_camera_ray(_addr(desc), float(row), float(col), use, dx, dy, _dp(m))
    return m


def camera_direction(desc, row, col):
    m = np.zeros(4)
    lib().oracle_camera_direction(_addr(desc), float(row), float(col), _dp(m))
    return m


def inner_product(desc, position, v, w):
    p, a, b = (np.ascontiguousarray(x, np.float64) for x in (position, v, w))
    return lib().oracle_inner_product(_addr(desc), _dp(p), _dp(a), _dp(b))


def stratified_offset(row, col, sr, sc, n):
    dx, dy = C.c_double(), C.c_double()
    lib().oracle_stratified_offset(row, col, sr, sc, n, C.byref(dx), C.byref(dy))
    return dx.value, dy.value


def blend(self_c, other):
    a, b, o = np.ascontiguousarray(self_c, np.float64), np.ascontiguousarray(other, np.float64), np.zeros(4)
    lib().oracle_blend(_dp(a), _dp(b), _dp(o))
    return o


def texture_color(desc, obj, u, v, redshift, temperature):
    o = np.zeros(4)
    lib().oracle_texture_color(_addr(desc), obj, u, v, redshift, temperature, _dp(o))
    return o


def killing_coefficients(r_s, a, r):
    ut, up = C.c_double(), C.c_double()
    rc = lib().oracle_killing_coefficients(r_s, a, r, C.byref(ut), C.byref(up))
    return rc, ut.value, up.value


def object_intersects(desc, obj, a, b):
    pa, pb = np.ascontiguousarray(a, np.float64), np.ascontiguousarray(b, np.float64)
    pt, t = np.zeros(4), C.c_double()
    hit = lib().oracle_object_intersects(_addr(desc), obj, _dp(pa), _dp(pb), _dp(pt), C.byref(t))
    return bool(hit), pt, t.value


def xyz_to_srgb8(xyza, tone: int, exposure: float = 1.0):
    """color.rs:204-298 output stage: (n,4) f64 XYZA -> (n,3) u8 sRGB."""
    x = np.ascontiguousarray(xyza, np.float64).reshape(-1, 4)
    out = np.zeros((x.shape[0], 3), np.uint8)
    lib().oracle_xyz_to_srgb8(_dp(x), x.shape[0], tone, exposure, out.ctypes.data_as(_u8p))
    return out


# ---- VolumetricDisc pieces (volumetric_disc.rs) ----
def perlin_table(seed: int) -> np.ndarray:
    out = np.zeros(256, np.uint8)
    lib().oracle_perlin_table(seed, out.ctypes.data_as(_u8p))
    return out


def perlin(seed: int, x: float, y: float, z: float) -> float:
    return lib().oracle_perlin(seed, x, y, z)


def vdisc_density(desc, obj: int, p) -> float:
    return lib().oracle_vdisc_density(_addr(desc), obj, _dp(np.asarray(p, np.float64)))


def vdisc_raymarch(desc, obj: int, ro, rd, freq=(1.0, 1.0, 0.0), cached=True):
    out = np.zeros(4)
    n = C.c_uint64()
    err = lib().oracle_vdisc_raymarch(_addr(desc), obj, _dp(np.asarray(ro, np.float64)),
                                      _dp(np.asarray(rd, np.float64)), _dp(np.asarray(freq, np.float64)),
                                      1 if cached else 0, _dp(out), C.byref(n))
    return err, out, n.value


# ---- geometry probes (the reference's unit tests, tests/test_reference_kats.py) ----
def _v(x, n=4):
    return np.ascontiguousarray(x, np.float64).reshape(n)


def should_stop(desc, y, i):
    return lib().oracle_should_stop(_addr(desc), _dp(_v(y, 8)), i)


def inside_horizon(desc, pos):
    return bool(lib().oracle_inside_horizon(_addr(desc), _dp(_v(pos))))


def radial_coordinate(desc, pos, cartesian=False):
    return lib().oracle_radial_coordinate(_addr(desc), _dp(_v(pos)), 1 if cartesian else 0)


def to_cartesian(desc, pos):
    out = np.zeros(4)
    lib().oracle_to_cartesian(_addr(desc), _dp(_v(pos)), _dp(out))
    return out


def stationary_velocity(desc, pos):
    out = np.zeros(4)
    lib().oracle_stationary_velocity(_addr(desc), _dp(_v(pos)), _dp(out))
    return out


def circular_orbit_velocity(desc, pos):
    out = np.zeros(4)
    err = lib().oracle_circular_orbit_velocity(_addr(desc), _dp(_v(pos)), _dp(out))
    return err, out


def geodesic_rhs(desc, pos, mom, y=None):
    """(initial state y0, RHS at y (default y0), momentum_from_state at y) of the ray's solver."""
    y0, rhs, p = np.zeros(8), np.zeros(8), np.zeros(4)
    yi = None if y is None else _v(y, 8)
    lib().oracle_geodesic_rhs(_addr(desc), _dp(_v(pos)), _dp(_v(mom)), _dp(yi) if yi is not None else None,
                              _dp(y0), _dp(rhs), _dp(p))
    return y0, rhs, p


def ks_metric(radius, a, x, y, z, contravariant=False):
    g = np.zeros(16)
    lib().oracle_ks_metric(radius, a, x, y, z, 1 if contravariant else 0, _dp(g))
    return g.reshape(4, 4)


def bl_metric(r_s, a, r, theta):
    g = np.zeros(16)
    lib().oracle_bl_metric(r_s, a, r, theta, _dp(g))
    return g.reshape(4, 4)


def redshift_static(desc, pos, mom, observer_energy):
    return lib().oracle_redshift_static(_addr(desc), _dp(_v(pos)), _dp(_v(mom)), observer_energy)


def should_supersample_pair(p, pc, q, qc, adaptive, min_lum):
    return bool(lib().oracle_should_supersample_pair(_dp(_v(p)), pc, _dp(_v(q)), qc,
                                                     C.cast(C.pointer(adaptive), C.c_void_p), min_lum))


def kerr_bl_rhs(r_s, a, e, l_z, q, y):
    out = np.zeros(8)
    lib().oracle_kerr_bl_rhs(r_s, a, e, l_z, q, _dp(_v(y, 8)), _dp(out))
    return out

