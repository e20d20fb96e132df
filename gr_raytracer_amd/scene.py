"""Host-side mirror of the reference's scene/render surface, over the C ABI.

Names follow mdreem/gr_raytracer:
  * GlobalOpts                 src/cli/cli.rs:5-47
  * load_scene                 main.rs:74-116 + cli/<geometry>.rs + cli/shared.rs:131-321
  * Scene.render_section       Raytracer::render_section_to_cie_buffer (raytracer.rs:177-318)
  * Scene.render_pixels        render_section_to_cie_buffer_raw (raytracer.rs:195-244)
  * Scene.color_of_ray         Scene::color_of_ray (scene.rs:114-220) for one camera pixel
  * SceneBuilder               scene.rs::test_scene::create_scene_with_camera (scene.rs:250-369)
Every call runs the HIP kernels in libgrt.so; there is no CPU path here.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from pathlib import Path
from typing import Optional, Sequence

import numpy as np

from . import _lib as L


# ------------------------------------------------------------------ options -------
@dataclass
class GlobalOpts:
    """clap GlobalOpts (cli.rs:5-47) with the reference defaults."""
    width: int = 500
    height: int = 500
    step_size: float = 0.01
    max_steps: int = 20000
    max_radius: float = 15000.0
    epsilon: float = 0.00001
    camera_position: Sequence[float] = (18.0, 0.0, 0.8)
    phi: float = 0.0
    theta: float = 0.0
    psi: float = 0.0
    tone_mapping: str = "reinhard"
    show_sampling_mask: bool = False
    sampling_mask_color: Sequence[int] = (255, 0, 255)

    def to_c(self) -> L.GlobalOpts:
        o = L.GlobalOpts()
        L.lib().grt_default_global_opts(C.byref(o))
        o.width, o.height = int(self.width), int(self.height)
        o.step_size, o.max_steps, o.max_radius = float(self.step_size), int(self.max_steps), float(self.max_radius)
        o.epsilon = float(self.epsilon)
        for k in range(3):
            o.camera_position[k] = float(self.camera_position[k])
            o.sampling_mask_color[k] = int(self.sampling_mask_color[k])
        o.phi, o.theta, o.psi = float(self.phi), float(self.theta), float(self.psi)
        o.tone_mapping = {"reinhard": 0, "global-linear": 1}[self.tone_mapping]
        o.show_sampling_mask = int(bool(self.show_sampling_mask))
        return o


def default_adaptive() -> L.AdaptiveConfig:
    c = L.AdaptiveConfig()
    L.lib().grt_default_adaptive_config(C.byref(c))
    return c


def device_count() -> int:
    return int(L.lib().grt_device_count())


# ------------------------------------------------------------------ scenes --------
class HostScene:
    """A TOML scene built on the host (textures decoded, camera tetrad, LUTs)."""

    def __init__(self, config_file: str, opts: GlobalOpts, resource_root: Optional[str] = None):
        self._h = C.c_void_p()
        rr = None if resource_root is None else str(resource_root).encode()
        L.check(L.lib().grt_host_scene_load(str(config_file).encode(), rr, C.byref(opts.to_c()), C.byref(self._h)),
                f"load_scene({config_file})")
        self.opts = opts

    @property
    def desc(self) -> L.SceneDesc:
        return L.lib().grt_host_scene_desc(self._h).contents

    def desc_ptr(self):
        return L.lib().grt_host_scene_desc(self._h)

    @property
    def info_log(self) -> list:
        """The reference's info-level lines of the scene setup, in order (grt_host_scene_log:
        the temperature LUT's, temperature.rs:55-102)."""
        return [x for x in (L.lib().grt_host_scene_log(self._h) or b"").decode().split("\n") if x]

    @property
    def adaptive(self) -> L.AdaptiveConfig:
        c = L.AdaptiveConfig()
        L.lib().grt_host_scene_adaptive(self._h, C.byref(c))
        return c

    def close(self) -> None:
        if self._h:
            L.lib().grt_host_scene_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load_scene(config_file: str, opts: Optional[GlobalOpts] = None, resource_root: Optional[str] = None) -> "Scene":
    """Parse a scene TOML + options and upload it (main.rs:74-116, cli/shared.rs:131-321)."""
    hs = HostScene(config_file, opts or GlobalOpts(), resource_root)
    return Scene(hs.desc_ptr(), keepalive=hs, adaptive=hs.adaptive)


@dataclass
class RenderResult:
    xyza: np.ndarray                 # float32 (n, 4)
    ray_class: np.ndarray            # uint8 (n,)
    status: np.ndarray               # uint8 (n,)
    xyza64: Optional[np.ndarray] = None
    steps: Optional[np.ndarray] = None
    stop_reason: Optional[np.ndarray] = None
    hits: Optional[np.ndarray] = None  # uint32 (n,): windows with an intersection (scene.rs:141-152)
    stats: dict = field(default_factory=dict)


@dataclass
class SectionResult:
    xyza64: np.ndarray          # float64 (n, 4)
    ray_class: np.ndarray       # uint8 (n,)
    status: np.ndarray          # uint8 (n,): the 1-spp ray's status
    n_supersampled: int
    stats: dict
    n_failed_subsamples: int
    failed_subsamples: np.ndarray  # (m, 3) uint32: section pixel, stratum, status (m <= capacity)
    # log_events=True: the 1-spp rays' stop reasons and accepted steps, and the supersample
    # sub-rays that ended on NaN coordinates or without a terminal event (no error):
    # (k, 4) uint32 section pixel, stratum, stop reason, accepted steps (scene.rs:178-202)
    stop: Optional[np.ndarray] = None
    steps: Optional[np.ndarray] = None
    subsample_events: Optional[np.ndarray] = None


def _stats_dict(st: L.Stats) -> dict:
    return {"accepted_steps": int(st.accepted_steps), "attempts": int(st.attempts), "rays": int(st.rays),
            "hit_overflows": int(st.hit_overflows), "kernel_ms": float(st.kernel_ms),
            "march_jobs": int(st.march_jobs), "march_samples": int(st.march_samples),
            "march_noise_samples": int(st.march_noise_samples), "march_emit_samples": int(st.march_emit_samples)}


class Scene:
    """Device-resident scene (grt_scene); one device copy per GPU, created lazily."""

    def __init__(self, desc_ptr, keepalive=None, adaptive: Optional[L.AdaptiveConfig] = None):
        self._s = C.c_void_p()
        L.check(L.lib().grt_scene_create(desc_ptr, C.byref(self._s)), "grt_scene_create")
        self._keep = keepalive
        self.desc = desc_ptr.contents
        self.adaptive = adaptive if adaptive is not None else default_adaptive()

    @property
    def rows(self) -> int:
        return int(self.desc.camera.rows)

    @property
    def cols(self) -> int:
        return int(self.desc.camera.cols)

    def close(self) -> None:
        if self._s:
            L.lib().grt_scene_destroy(self._s)
            self._s = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render_pixels(self, row0: int = 0, col0: int = 0, rows: Optional[int] = None, cols: Optional[int] = None,
                      device: int = 0, offsets=None, aux: bool = True) -> RenderResult:
        """1-spp trace of a rectangle, or of an offset list (pixel_index, dx, dy)."""
        rows = self.rows - row0 if rows is None else rows
        cols = self.cols - col0 if cols is None else cols
        off = None
        keep = []
        if offsets is not None:
            pix, dx, dy = (np.ascontiguousarray(offsets[0], np.uint32), np.ascontiguousarray(offsets[1], np.float64),
                           np.ascontiguousarray(offsets[2], np.float64))
            keep += [pix, dx, dy]
            off = L.Offsets(len(pix), L.ptr(pix, C.c_uint32), L.dptr(dx), L.dptr(dy))
            n = len(pix)
        else:
            n = rows * cols
        xyza = np.zeros((n, 4), np.float32)
        cls = np.zeros(n, np.uint8)
        status = np.zeros(n, np.uint8)
        res = RenderResult(xyza, cls, status)
        a = None
        if aux:
            res.xyza64 = np.zeros((n, 4), np.float64)
            res.steps = np.zeros(n, np.uint32)
            res.stop_reason = np.zeros(n, np.uint8)
            res.hits = np.zeros(n, np.uint32)
            a = L.AuxOut(L.dptr(res.xyza64), L.ptr(res.steps, C.c_uint32), L.ptr(res.stop_reason, C.c_uint8),
                         L.ptr(res.hits, C.c_uint32))
        st = L.Stats()
        L.check(L.lib().grt_render_pixels(self._s, device, row0, col0, rows, cols,
                                          C.byref(off) if off is not None else None,
                                          L.ptr(xyza, C.c_float), L.ptr(cls, C.c_uint8), L.ptr(status, C.c_uint8),
                                          C.byref(a) if a is not None else None, C.byref(st)), "grt_render_pixels")
        res.stats = _stats_dict(st)
        return res

    def render_shard(self, band_rows: int, shard: int, n_shards: int, device: int = 0,
                     aux: bool = True) -> RenderResult:
        """The local rows of one cyclic row-band shard (grt_render_shard), full width."""
        sh = L.RowShard(band_rows, shard, n_shards)
        n = int(L.lib().grt_shard_row_count(self.rows, C.byref(sh))) * self.cols
        xyza, cls, status = np.zeros((n, 4), np.float32), np.zeros(n, np.uint8), np.zeros(n, np.uint8)
        res = RenderResult(xyza, cls, status)
        a = None
        if aux:
            res.xyza64, res.steps, res.stop_reason = np.zeros((n, 4)), np.zeros(n, np.uint32), np.zeros(n, np.uint8)
            res.hits = np.zeros(n, np.uint32)
            a = L.AuxOut(L.dptr(res.xyza64), L.ptr(res.steps, C.c_uint32), L.ptr(res.stop_reason, C.c_uint8),
                         L.ptr(res.hits, C.c_uint32))
        st = L.Stats()
        L.check(L.lib().grt_render_shard(self._s, device, C.byref(sh), L.ptr(xyza, C.c_float), L.ptr(cls, C.c_uint8),
                                         L.ptr(status, C.c_uint8), C.byref(a) if a is not None else None,
                                         C.byref(st)), "grt_render_shard")
        res.stats = _stats_dict(st)
        return res

    def render_frame_multi(self, devices=(0,), band_rows: int = 16, adaptive: Optional[L.AdaptiveConfig] = None,
                           supersample: bool = False, sampling_mask_xyza=None, fields=("xyza", "class", "status"),
                           fail_capacity: int = 0) -> dict:
        """The whole frame over `devices` (grt_render_frame_multi: cyclic row bands, one host
        thread per device, one RCCL gather to devices[0]).  fields: which of "xyza" (f32),
        "xyza64", "class", "status", "stop", "steps" to return (frame order).  supersample:
        the adaptive pass with `adaptive` (default: the scene's own configuration).
        Returns a dict of the fields plus "stats", "n_supersampled", "report" and, with
        fail_capacity, "failures" (pixel, sample, status, stop, steps arrays)."""
        n = self.rows * self.cols
        want = set(fields)
        arrays = {}
        if "xyza" in want:
            arrays["xyza"] = np.zeros((n, 4), np.float32)
        if "xyza64" in want or supersample or sampling_mask_xyza is not None:
            arrays["xyza64"] = np.zeros((n, 4), np.float64)
        for k, dt in (("class", np.uint8), ("status", np.uint8), ("stop", np.uint8), ("steps", np.uint32)):
            if k in want:
                arrays[k] = np.zeros(n, dt)
        out = L.FrameOut(L.ptr(arrays["xyza"], C.c_float) if "xyza" in arrays else None,
                         L.dptr(arrays["xyza64"]) if "xyza64" in arrays else None,
                         L.ptr(arrays["class"], C.c_uint8) if "class" in arrays else None,
                         L.ptr(arrays["status"], C.c_uint8) if "status" in arrays else None,
                         L.ptr(arrays["stop"], C.c_uint8) if "stop" in arrays else None,
                         L.ptr(arrays["steps"], C.c_uint32) if "steps" in arrays else None)
        cfg = None
        if supersample or sampling_mask_xyza is not None:
            cfg = L.AdaptiveConfig()
            C.memmove(C.byref(cfg), C.byref(adaptive if adaptive is not None else self.adaptive), C.sizeof(cfg))
            cfg.enabled = 1 if supersample else cfg.enabled
        mask = None
        if sampling_mask_xyza is not None:
            mask = np.ascontiguousarray(sampling_mask_xyza, np.float64)
        devs = (C.c_int * len(devices))(*devices)
        fails = None
        farr = {}
        if fail_capacity:
            farr = {"pixel": np.zeros(fail_capacity, np.uint32), "sample": np.zeros(fail_capacity, np.uint32),
                    "status": np.zeros(fail_capacity, np.uint8), "stop": np.zeros(fail_capacity, np.uint8),
                    "steps": np.zeros(fail_capacity, np.uint32)}
            fails = L.SubsampleFailures(fail_capacity, L.ptr(farr["pixel"], C.c_uint32),
                                        L.ptr(farr["sample"], C.c_uint32), L.ptr(farr["status"], C.c_uint8), 0,
                                        L.ptr(farr["stop"], C.c_uint8), L.ptr(farr["steps"], C.c_uint32))
        nsel = C.c_uint64(0)
        st = L.Stats()
        rep = L.MultiReport()
        L.check(L.lib().grt_render_frame_multi(self._s, len(devices), devs, band_rows,
                                               C.byref(cfg) if cfg is not None else None,
                                               L.dptr(mask) if mask is not None else None, C.byref(out),
                                               C.byref(nsel), C.byref(st), C.byref(fails) if fails is not None else None,
                                               C.byref(rep)), "grt_render_frame_multi")
        arrays["stats"] = _stats_dict(st)
        arrays["n_supersampled"] = int(nsel.value)
        arrays["report"] = rep
        if fails is not None:
            m = min(int(fails.count), fail_capacity)
            arrays["failures"] = {k: v[:m] for k, v in farr.items()}
            arrays["failures"]["count"] = int(fails.count)
        return arrays

    def render_section(self, from_row: int = 0, from_col: int = 0, to_row: Optional[int] = None,
                       to_col: Optional[int] = None, adaptive: Optional[L.AdaptiveConfig] = None,
                       sampling_mask_xyza=None, device: int = 0):
        """render_section_to_cie_buffer (raytracer.rs:177-318): f64 XYZA per pixel.
        Returns (xyza64, class, n_supersampled, stats)."""
        r = self.render_section_ex(from_row, from_col, to_row, to_col, adaptive, sampling_mask_xyza, device)
        return r.xyza64, r.ray_class, r.n_supersampled, r.stats

    def render_section_ex(self, from_row: int = 0, from_col: int = 0, to_row: Optional[int] = None,
                          to_col: Optional[int] = None, adaptive: Optional[L.AdaptiveConfig] = None,
                          sampling_mask_xyza=None, device: int = 0, failure_capacity: int = 1 << 16,
                          log_events: bool = False):
        """render_section plus each pixel's 1-spp status and the failed supersample
        sub-rays ((pixel, stratum, status), sorted; raytracer.rs:232-239, :357-362); with
        log_events, also what color_of_ray's NaN / no-terminal-event log lines need."""
        to_row = self.rows if to_row is None else to_row
        to_col = self.cols if to_col is None else to_col
        n = (to_row - from_row) * (to_col - from_col)
        out = np.zeros((n, 4), np.float64)
        cls = np.zeros(n, np.uint8)
        status = np.zeros(n, np.uint8)
        nsel = C.c_uint64(0)
        st = L.Stats()
        mask = None
        if sampling_mask_xyza is not None:
            mask = np.ascontiguousarray(sampling_mask_xyza, np.float64)
        fp = np.zeros(failure_capacity, np.uint32)
        fs = np.zeros(failure_capacity, np.uint32)
        fst = np.zeros(failure_capacity, np.uint8)
        fsp = np.zeros(failure_capacity, np.uint8)
        fn = np.zeros(failure_capacity, np.uint32)
        fails = L.SubsampleFailures(failure_capacity, L.ptr(fp, C.c_uint32), L.ptr(fs, C.c_uint32),
                                    L.ptr(fst, C.c_uint8), 0, L.ptr(fsp, C.c_uint8) if log_events else None,
                                    L.ptr(fn, C.c_uint32) if log_events else None)
        stop = np.zeros(n, np.uint8) if log_events else None
        steps = np.zeros(n, np.uint32) if log_events else None
        L.check(L.lib().grt_render_section_ex(self._s, device, from_row, from_col, to_row, to_col,
                                              C.byref(adaptive or self.adaptive),
                                              L.dptr(mask) if mask is not None else None, L.dptr(out),
                                              L.ptr(cls, C.c_uint8), C.byref(nsel), C.byref(st),
                                              L.ptr(status, C.c_uint8), C.byref(fails),
                                              L.ptr(stop, C.c_uint8) if log_events else None,
                                              L.ptr(steps, C.c_uint32) if log_events else None),
                "grt_render_section_ex")
        m = min(int(fails.count), failure_capacity)
        rows = np.stack([fp[:m], fs[:m], fst[:m].astype(np.uint32)], axis=1)
        if not log_events:
            return SectionResult(out, cls, status, int(nsel.value), _stats_dict(st), int(fails.count), rows)
        failed = fst[:m] != 0
        events = np.stack([fp[:m], fs[:m], fsp[:m].astype(np.uint32), fn[:m]], axis=1)[~failed]
        return SectionResult(out, cls, status, int(nsel.value), _stats_dict(st), int(fails.count) - len(events),
                             rows[failed], stop, steps, events)

    def _trace(self, fn, a, b, width: int, capacity: int, device: int):
        a = np.ascontiguousarray(a, np.float64).reshape(-1, width)
        b = np.ascontiguousarray(b, np.float64).reshape(-1, width)
        n = a.shape[0]
        steps = np.zeros((n, capacity, 9), np.float64)
        n_steps = np.zeros(n, np.uint64)
        stop, status = np.zeros(n, np.uint8), np.zeros(n, np.uint8)
        L.check(fn(self._s, device, n, L.dptr(a), L.dptr(b), capacity, L.dptr(steps), L.ptr(n_steps, C.c_uint64),
                   L.ptr(stop, C.c_uint8), L.ptr(status, C.c_uint8)), "grt_trace")
        return Trajectories(steps, n_steps.astype(np.int64), stop, status)

    def trace_pixels(self, rows, cols, capacity: Optional[int] = None, device: int = 0) -> "Trajectories":
        """Whole trajectories of camera rays (Raytracer::integrate_ray_at_point,
        raytracer.rs:499-507; `render-ray`).  capacity defaults to max_steps records."""
        cap = int(self.desc.max_steps) if capacity is None else capacity
        return self._trace(L.lib().grt_trace_pixels, np.atleast_1d(rows), np.atleast_1d(cols), 1, cap, device)

    def trace_rays(self, positions, momenta, capacity: Optional[int] = None, device: int = 0) -> "Trajectories":
        """Whole trajectories from native-chart positions / contravariant momenta (n x 4)."""
        cap = int(self.desc.max_steps) if capacity is None else capacity
        return self._trace(L.lib().grt_trace_rays, positions, momenta, 4, cap, device)

    def color_of_ray(self, row: int, col: int, device: int = 0):
        """Colour, class and status of one camera pixel (Scene::color_of_ray)."""
        r = self.render_pixels(row, col, 1, 1, device=device)
        return r.xyza64[0], int(r.ray_class[0]), int(r.status[0])

    def health(self, row0: int = 0, col0: int = 0, rows: Optional[int] = None, cols: Optional[int] = None,
               device: int = 0, per_ray: bool = False) -> dict:
        """The reference's invariant monitors over a rectangle (grt_health_pixels): camera-ray
        null condition (scene.rs:116-124) and k.k / constants-of-motion drifts
        (integrator.rs:91-201).  per_ray adds an (n, 5) array: |k.k| at the camera, largest
        |k.k| along the path, largest drift of E, L_z, Q."""
        rows = self.rows - row0 if rows is None else rows
        cols = self.cols - col0 if cols is None else cols
        h = L.Health()
        arr = np.zeros((rows * cols, 5)) if per_ray else None
        L.check(L.lib().grt_health_pixels(self._s, device, row0, col0, rows, cols, C.byref(h),
                                          L.ptr(arr, C.c_double) if per_ray else None), "grt_health_pixels")
        nc = h.n_constants
        out = {"rays": h.rays, "failed": h.failed, "null_violations": h.null_violations, "max_null": h.max_null,
               "kk_drift_rays": h.kk_drift_rays, "max_kk_drift": h.max_kk_drift, "n_constants": nc,
               "constant_drift_rays": list(h.constant_drift_rays)[:nc],
               "max_constant_drift": list(h.max_constant_drift)[:nc]}
        if per_ray:
            out["per_ray"] = arr
        return out

    def tail_handoffs(self, device: int = 0) -> int:
        """Rays the last Kerr-Schild trace on `device` handed to the tail kernel."""
        n = C.c_uint64()
        L.check(L.lib().grt_tail_handoffs(self._s, device, C.byref(n)), "grt_tail_handoffs")
        return n.value

    def tail_report(self, device: int = 0, capacity: int = 0) -> dict:
        """Hand-off diagnostics of the last Kerr-Schild trace: count, timeline (s since the
        integrate kernel started) and the handed-off rays' output slots and step counts."""
        n = C.c_uint64()
        tl = (C.c_double * 3)()
        slot = np.zeros(capacity, np.uint64)
        step = np.zeros(capacity, np.uint64)
        L.check(L.lib().grt_tail_report(self._s, device, C.byref(n), tl, L.ptr(slot, C.c_uint64),
                                        L.ptr(step, C.c_uint64), capacity), "grt_tail_report")
        k = min(n.value, capacity)
        return {"handed_off": n.value, "drained_s": tl[0], "handoff_s": tl[1], "tail_end_s": tl[2],
                "slot": slot[:k], "step": step[:k]}


def set_two_ended(on: bool = True) -> None:
    """Probe-ordered traces take the tile queue from both ends (grt_set_two_ended): the
    priority wave of each SIMD the longest tiles, the others the shortest.  Scheduling
    only; results are identical in both modes."""
    L.check(L.lib().grt_set_two_ended(1 if on else 0), "grt_set_two_ended")


ARITH_EXACT, ARITH_FUSED = 0, 1


def set_arithmetic(mode) -> None:
    """grt_set_arithmetic: "exact" / 0 (the reference's roundings, default) or "fused" / 1
    (FMA contraction in the light charts' kernels; Kerr-Schild stays exact)."""
    m = {"exact": 0, "fused": 1}.get(mode, mode)
    L.check(L.lib().grt_set_arithmetic(int(m)), "grt_set_arithmetic")


def get_arithmetic() -> int:
    return int(L.lib().grt_get_arithmetic())


def set_tail(threshold: int = -1) -> None:
    """Long-ray hand-off of Kerr-Schild traces (grt_set_tail): -1 auto, 0 off, > 0 the
    live-ray threshold.  Scheduling only; results are identical in every mode."""
    L.check(L.lib().grt_set_tail(int(threshold)), "grt_set_tail")


# --------------------------------------------------------- programmatic scenes ----
@dataclass
class Checker:
    """CheckerMapper (texture.rs:212-257)."""
    beaming_exponent: float
    width: float
    height: float
    color1: Sequence[int]
    color2: Sequence[int]


@dataclass
class Bitmap:
    """TextureMapper (texture.rs:41-102): RGBA8 array (H, W, 4)."""
    beaming_exponent: float
    rgba: np.ndarray


@dataclass
class BlackBody:
    """BlackBodyMapper (texture.rs:104-210)."""
    beaming_exponent: float = 0.0


def srgb_to_xyza(r: int, g: int, b: int, a: int = 255) -> np.ndarray:
    out = np.zeros(4, np.float64)
    L.lib().grt_srgb_to_xyza(r, g, b, a, L.dptr(out))
    return out


def xyz_to_srgb8(xyza, tone_mapping: int = 0, exposure: float = 1.0, device: Optional[int] = None) -> np.ndarray:
    """Output stage (color.rs:204-298): (n,4) f64 XYZA -> (n,3) u8 sRGB.  device=None
    runs the host C++ path (grt_xyz_to_srgb8), an ordinal runs the HIP kernels
    (grt_xyz_to_srgb8_device); both return the reference's bytes."""
    x = np.ascontiguousarray(xyza, np.float64).reshape(-1, 4)
    out = np.zeros((x.shape[0], 3), np.uint8)
    if device is None:
        L.check(L.lib().grt_xyz_to_srgb8(L.dptr(x), x.shape[0], tone_mapping, exposure, L.ptr(out, C.c_uint8)),
                "grt_xyz_to_srgb8")
    else:
        L.check(L.lib().grt_xyz_to_srgb8_device(device, L.dptr(x), x.shape[0], tone_mapping, exposure,
                                                 L.ptr(out, C.c_uint8)), "grt_xyz_to_srgb8_device")
    return out


@dataclass
class Trajectories:
    """steps[k, i] = (t, x^0..x^3, p^0..p^3) of ray k's step i, i < min(n_steps[k], capacity)."""
    steps: np.ndarray
    n_steps: np.ndarray
    stop_reason: np.ndarray
    status: np.ndarray

    def ray(self, k: int) -> np.ndarray:
        return self.steps[k, : min(int(self.n_steps[k]), self.steps.shape[1])]


def ray_at(geometry: int, radius: float, a: float, position, direction):
    """render_ray_at's initial (position, momentum) in the geometry's chart (grt_ray_at)."""
    p, d = np.ascontiguousarray(position, np.float64), np.ascontiguousarray(direction, np.float64)
    po, mo = np.zeros(4), np.zeros(4)
    L.check(L.lib().grt_ray_at(geometry, radius, a, L.dptr(p), L.dptr(d), L.dptr(po), L.dptr(mo)), "grt_ray_at")
    return po, mo


def write_trajectory_csv(path: str, geometry: int, a: float, records) -> None:
    """IntegratedRay::save (ray.rs:35-54) of (n, 9) records."""
    r = np.ascontiguousarray(records, np.float64).reshape(-1, 9)
    L.check(L.lib().grt_write_trajectory_csv(str(path).encode(), geometry, a, L.dptr(r), r.shape[0]),
            "grt_write_trajectory_csv")


def format_f64(v: float) -> str:
    """Rust's Display of an f64 (shortest round-trip digits, positional)."""
    buf = C.create_string_buffer(1200)
    L.lib().grt_format_f64(float(v), buf, 1200)
    return buf.value.decode()


def format_f64_debug(v: float) -> str:
    """Rust's Debug of an f64 ({:?}): Display's digits with ".0" on integral values, and
    exponential notation outside 1e-4 <= |v| < 1e16."""
    import math
    if math.isnan(v) or math.isinf(v):
        return format_f64(v)
    if v != 0.0 and (abs(v) < 1e-4 or abs(v) >= 1e16):
        m, e = repr(float(v)).lower().split("e") if "e" in repr(float(v)).lower() else (repr(float(v)), "0")
        return f"{m.rstrip('0').rstrip('.') if '.' in m else m}e{int(e)}"
    d = format_f64(v)
    return d if "." in d else d + ".0"


def coordinate_system_debug(geometry: int, a: float) -> str:
    """CoordinateSystem's Debug form for a geometry (geometry/*.rs coordinate_system, point.rs:11)."""
    if geometry in (L.GEOM_SCHWARZSCHILD, L.GEOM_EUCLIDEAN_SPHERICAL):
        return "Spherical"
    if geometry == L.GEOM_KERR_BL:
        return f"BoyerLindquist {{ a: {format_f64_debug(a)} }}"
    return "Cartesian"


def duration_debug_2(secs: float) -> str:
    """A Duration's Debug form with two decimals ({:.2?}): the largest of s / ms / us / ns
    with a non-zero integer part, the dropped digits rounded half up."""
    ns = int(round(secs * 1e9))
    for div, unit in ((10 ** 9, "s"), (10 ** 6, "ms"), (10 ** 3, "\u00b5s")):
        if ns >= div:
            h = (ns * 100 + div // 2) // div
            return f"{h // 100}.{h % 100:02d}{unit}"
    return f"{ns}.00ns"


def r_isco(radius: float, a: float) -> float:
    return float(L.lib().grt_r_isco(radius, a))


def blackbody_xyz(temperature: float, redshift: float = 1.0) -> np.ndarray:
    out = np.zeros(3, np.float64)
    L.lib().grt_blackbody_xyz(temperature, redshift, L.dptr(out))
    return out


def kerr_temperature_lut(temperature: float, outer_radius: float, a: float, radius: float, n: int = 1000):
    lr, lt, ri = np.zeros(n), np.zeros(n), C.c_double(0.0)
    L.check(L.lib().grt_kerr_temperature_lut(temperature, outer_radius, a, radius, n, L.dptr(lr), L.dptr(lt),
                                             C.byref(ri)), "KerrTemperatureComputer::new")
    return lr, lt, float(ri.value)


def cartesian_to_spherical(p) -> np.ndarray:
    i, o = np.ascontiguousarray(p, np.float64), np.zeros(4)
    L.lib().grt_cartesian_to_spherical(L.dptr(i), L.dptr(o))
    return o


def cartesian_to_boyer_lindquist(a: float, p) -> np.ndarray:
    i, o = np.ascontiguousarray(p, np.float64), np.zeros(4)
    L.lib().grt_cartesian_to_boyer_lindquist(a, L.dptr(i), L.dptr(o))
    return o


def build_camera(geometry: int, radius: float, a: float, position, velocity, alpha: float, rows: int, cols: int,
                 phi: float = 0.0, theta: float = 0.0, psi: float = 0.0) -> L.CameraDesc:
    """Camera::new (camera.rs:151-196)."""
    cam = L.CameraDesc()
    p, v = np.ascontiguousarray(position, np.float64), np.ascontiguousarray(velocity, np.float64)
    L.check(L.lib().grt_camera_build(geometry, radius, a, L.dptr(p), L.dptr(v), alpha, rows, cols, phi, theta, psi,
                                     C.byref(cam)), "Camera::new")
    return cam


def stationary_velocity(geometry: int, radius: float, a: float, position) -> np.ndarray:
    p, o = np.ascontiguousarray(position, np.float64), np.zeros(4)
    L.lib().grt_stationary_velocity(geometry, radius, a, L.dptr(p), L.dptr(o))
    return o


class SceneBuilder:
    """Assemble a grt_scene_desc in Python, as the reference tests do with
    `create_scene_with_camera` (scene.rs:281-369)."""

    def __init__(self, geometry: int, radius: float = 0.0, a: float = 0.0, horizon_epsilon: float = 0.0):
        self.d = L.SceneDesc()
        self.d.abi_version = L.GRT_ABI_VERSION
        self.d.geometry, self.d.radius, self.d.a, self.d.horizon_epsilon = geometry, radius, a, horizon_epsilon
        self.d.object_hit_opacity_threshold = 0.5
        self._fill_srgb()
        self._keep = []
        self._need_bb = False

    def _fill_srgb(self):
        # inv_compand_srgb (color.rs:301-308) of each 8-bit code; math.pow is the C libm pow
        for i in range(256):
            u = i / 255.0
            self.d.srgb_to_linear[i] = u / 12.92 if u <= 0.04045 else math.pow((u + 0.055) / 1.055, 2.4)

    def integration(self, max_steps: int, max_radius: float, step_size: float, epsilon: float) -> "SceneBuilder":
        self.d.max_steps, self.d.max_radius, self.d.step_size, self.d.epsilon = max_steps, max_radius, step_size, epsilon
        return self

    def camera(self, position, velocity, alpha: float, rows: int, cols: int, phi=0.0, theta=0.0, psi=0.0):
        self.d.camera = build_camera(self.d.geometry, self.d.radius, self.d.a, position, velocity, alpha, rows, cols,
                                     phi, theta, psi)
        return self

    def _texture(self, t) -> L.TextureDesc:
        d = L.TextureDesc()
        d.beaming_exponent = t.beaming_exponent
        if isinstance(t, Checker):
            d.kind = L.TEX_CHECKER
            d.checker_width, d.checker_height = t.width, t.height
            c1, c2 = srgb_to_xyza(*t.color1, 255), srgb_to_xyza(*t.color2, 255)
            c1[3] = c2[3] = 1.0
            for k in range(4):
                d.c1[k], d.c2[k] = c1[k], c2[k]
        elif isinstance(t, Bitmap):
            arr = np.ascontiguousarray(t.rgba, np.uint8)
            assert arr.ndim == 3 and arr.shape[2] == 4
            self._keep.append(arr)
            d.kind = L.TEX_BITMAP
            d.rgba = L.ptr(arr, C.c_uint8)
            d.height, d.width = arr.shape[0], arr.shape[1]
        else:
            d.kind = L.TEX_BLACKBODY
            self._need_bb = True
        return d

    def celestial(self, texture, temperature: float = 0.0) -> "SceneBuilder":
        self.d.celestial = self._texture(texture)
        self.d.celestial_temperature = temperature
        return self

    def add_sphere(self, radius: float, center, texture, temperature: float = 0.0) -> "SceneBuilder":
        o = self.d.objects[self.d.n_objects]
        o.kind, o.radius, o.temperature = L.OBJ_SPHERE, radius, temperature
        for k in range(3):
            o.center[k] = center[k]
        o.texture = self._texture(texture)
        self.d.n_objects += 1
        return self

    def add_disc(self, inner_radius: float, outer_radius: float, texture, temperature: float = 0.0,
                 constant_temperature: Optional[bool] = None) -> "SceneBuilder":
        """Disc with geometry.get_temperature_computer(temperature, inner, outer)."""
        o = self.d.objects[self.d.n_objects]
        o.kind, o.inner_radius, o.outer_radius = L.OBJ_DISC, inner_radius, outer_radius
        const = (self.d.geometry in (L.GEOM_EUCLIDEAN, L.GEOM_EUCLIDEAN_SPHERICAL) if constant_temperature is None
                 else constant_temperature)
        if const:
            o.temp_kind, o.temp_constant = L.TEMP_CONSTANT, temperature
        else:
            spin = 0.0 if self.d.geometry == L.GEOM_SCHWARZSCHILD else self.d.a
            lr, lt, ri = kerr_temperature_lut(temperature, outer_radius, spin, self.d.radius)
            self._keep += [lr, lt]
            o.temp_kind, o.r_isco, o.lut_n = L.TEMP_KERR_LUT, ri, len(lr)
            o.lut_r, o.lut_t = L.dptr(lr), L.dptr(lt)
        o.texture = self._texture(texture)
        self.d.n_objects += 1
        return self

    def add_volumetric_disc(self, inner_radius: float, outer_radius: float, texture, temperature: float = 0.0, *,
                            axis=(0.0, 0.0, 1.0), num_octaves: int = 8, perlin_seed: int = 1,
                            max_steps: int = 50000, step_size: float = 0.002, thickness: float = 0.1,
                            density_multiplier: float = 500.0, brightness_reference_temperature: float = 1000.0,
                            absorption: float = 0.3, scattering: float = 0.4, noise_scale=(1.0, 1.0, 1.0),
                            noise_offset: float = 0.0,
                            constant_temperature: Optional[bool] = None) -> "SceneBuilder":
        """VolumetricDisc::new (volumetric_disc.rs:43-95) with the Disc temperature model."""
        self.add_disc(inner_radius, outer_radius, texture, temperature, constant_temperature)
        o = self.d.objects[self.d.n_objects - 1]
        o.kind = L.OBJ_VOLUMETRIC_DISC
        for k in range(3):
            o.axis[k], o.noise_scale[k] = axis[k], noise_scale[k]
        o.num_octaves, o.perlin_seed, o.march_max_steps, o.march_step_size = num_octaves, perlin_seed, max_steps, step_size
        o.thickness, o.density_multiplier = thickness, density_multiplier
        o.brightness_reference_temperature = brightness_reference_temperature
        o.absorption, o.scattering, o.noise_offset = absorption, scattering, noise_offset
        return self

    def build(self) -> L.SceneDesc:
        if self._need_bb and not self.d.bb_n:
            lt, xyz = np.zeros(1000), np.zeros(3000)
            L.check(L.lib().grt_blackbody_lut(1000, L.dptr(lt), L.dptr(xyz)), "BlackBodyMapper::new")
            self._keep += [lt, xyz]
            self.d.bb_log_t, self.d.bb_xyz, self.d.bb_n = L.dptr(lt), L.dptr(xyz), 1000
        self.d._keepalive = self._keep  # type: ignore[attr-defined]
        return self.d

    def scene(self) -> Scene:
        d = self.build()
        return Scene(C.pointer(d), keepalive=(self, d))
