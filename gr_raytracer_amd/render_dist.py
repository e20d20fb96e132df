"""Multi-GPU `render`: the reference's `render` subcommand with the frame split across
the GPUs of a node (BASELINE config C4).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m gr_raytracer_amd.render_dist --width=4096 --height=4096 --max-steps=1000000 \\
        --camera-position=-10,0,-0.5 --theta=1.52 --psi=-1.57 --phi=0 \\
        --config-file scene-definitions/kerr.toml render --filename kerr.png

The flags are the reference's (cli.rs:5-113, the same set as the single-GPU `grt`
binary); `--resource-root DIR` resolves texture paths and `--raw-out FILE` dumps the
f64 XYZA frame, as in `grt`.  One process per GPU: rank r uses GPU LOCAL_RANK, traces
the cyclic row bands b with b % world == r, and the frame is assembled on rank 0 with
one RCCL gather (plus, for the stock TOMLs' adaptive supersampling, one allgather of
the 1-spp luminance, opacity and class; gr_raytracer_amd.distributed).  The pixels are
identical to a single-GPU `grt ... render` of the same scene.  Sections (--from-row ...)
are single-GPU only (use `grt`).  Without torchrun it runs as a world of one.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

RENDER_FLAGS = ("--filename", "--from-row", "--from-col", "--to-row", "--to-col")


# exit status of a frame written with pixels that lost hit candidates (the device hit pool
# could not hold them after two reserves): the image is incomplete
EXIT_INCOMPLETE = 3

# Debug names of the RaytracerError variants a pixel can end in (grt_main.cpp's table)
ERROR_NAMES = {1: "IntegrationError(MaxStepsReached)", 2: "NoCircularOrbitPossible", 3: "BelowRISCO",
               4: "NonFiniteRadius"}


def _log(msg: str) -> None:
    """One log line in one write(2): lines of ranks that share a stderr pipe do not interleave."""
    os.write(2, (msg + "\n").encode())


def log_ray_event(row: int, col: int, stop: int, accepted: int) -> None:
    """scene.rs:178-183 / :196-202 for an error-free ray that ended on NaN coordinates or
    without a terminal event (Ray's Debug form cut to its pixel; steps.len() = accepted + 1)."""
    if stop == 3:  # StopReason::CoordinateIsNan
        _log(f"[render_dist] ERROR Ray hit NaN coordinates: Ray {{ row: {row}, col: {col}, .. }} with {accepted + 1} "
              "steps.")
    elif stop == 0:  # no stop reason
        _log(f"[render_dist] ERROR Ray did not hit anything: Ray {{ row: {row}, col: {col}, .. }} at Some(Step {{ .. }}) "
              f"with {accepted + 1} steps.")


def _csv(n: int, conv=float):
    def parse(v: str):
        parts = v.split(",")
        if len(parts) != n:
            raise argparse.ArgumentTypeError(f"expected {n} comma-separated values, got {v!r}")
        return [conv(p) for p in parts]
    return parse


def _rgb(v: str):
    """impl FromStr for Color (color.rs:151-170): three trimmed u8 components."""
    parts = v.split(",")
    out = []
    for part in parts:
        t = part.strip()
        t = t[1:] if t.startswith("+") else t
        if not t or not t.isdigit() or not t.isascii() or int(t) > 255:
            raise argparse.ArgumentTypeError(f"invalid RGB color '{v}'; expected three values from 0 to 255")
        out.append(int(t))
    if len(out) != 3:
        raise argparse.ArgumentTypeError(f"invalid RGB color '{v}'; expected R,G,B (for example 255,0,255)")
    return out


def parse_args(argv):
    """cli.rs:5-113 for `render`: global options anywhere, then the subcommand."""
    p = argparse.ArgumentParser(prog="render_dist", description=__doc__.splitlines()[0])
    p.add_argument("--width", type=int, default=500)
    p.add_argument("--height", type=int, default=500)
    p.add_argument("--step-size", type=float, default=0.01)
    p.add_argument("--max-steps", type=int, default=20000)
    p.add_argument("--max-radius", type=float, default=15000.0)
    p.add_argument("--epsilon", type=float, default=0.00001)
    p.add_argument("--camera-position", type=_csv(3), default=[18.0, 0.0, 0.8])
    p.add_argument("--phi", type=float, default=0.0)
    p.add_argument("--theta", type=float, default=0.0)
    p.add_argument("--psi", type=float, default=0.0)
    p.add_argument("--tone-mapping", choices=["reinhard", "global-linear"], default="reinhard")
    p.add_argument("--show-sampling-mask", action="store_true")
    p.add_argument("--sampling-mask-color", type=_rgb, default=[255, 0, 255])
    p.add_argument("-c", "--config-file", required=True)
    p.add_argument("--resource-root", default=None)
    p.add_argument("--raw-out", default=None)
    p.add_argument("--band-rows", type=int, default=16, help="rows per cyclic band (not in the reference)")
    p.add_argument("--backend", default=None, help="torch.distributed backend (default nccl = RCCL)")
    p.add_argument("action", choices=["render"])
    p.add_argument("--filename", default="render.png")
    for f in RENDER_FLAGS[1:]:
        p.add_argument(f, type=int, default=None)
    a = p.parse_args(argv)
    if any(getattr(a, f[2:].replace("-", "_")) is not None for f in RENDER_FLAGS[1:]):
        p.error("sections (--from-row/--from-col/--to-row/--to-col) are single-GPU only: use grt")
    return a


def trace_until_complete(render_once, lost_pixels, grow_pool, log, attempts: int = 3):
    """Trace the frame until no pixel lost hit candidates, at most `attempts` times.

    render_once() traces the frame and returns its result; lost_pixels() returns the
    number of pixels that lost candidates in that trace, summed over every rank (the same
    value on each rank, so every rank takes the same branch); grow_pool() grows this
    rank's device hit pool from the trace's measured need (grt_hit_pool_reserve).
    Returns (result of the last trace, pixels still incomplete after it: 0 or the count)."""
    out = None
    for attempt in range(attempts):
        out = render_once()
        lost = lost_pixels()
        if lost == 0:
            return out, 0
        if attempt == attempts - 1:  # the pool cannot hold them (2^31 records): the frame is incomplete
            log(f"ERROR {lost} pixels lost hit candidates after growing the device hit pool {attempts - 1} "
                f"times; they are written without their candidates past the first 16, and the exit status "
                f"is {EXIT_INCOMPLETE}")
            return out, lost
        log(f"WARN {lost} pixels lost hit candidates (device hit pool full); growing the pool and tracing again")
        grow_pool()
    return out, 0


def exit_status(incomplete: int) -> int:
    """Process exit status of a rank: EXIT_INCOMPLETE when the written frame lacks candidates."""
    return EXIT_INCOMPLETE if incomplete else 0


def main(argv=None) -> int:
    a = parse_args(sys.argv[1:] if argv is None else argv)
    t_start = time.perf_counter()
    import ctypes as C

    import numpy as np
    import torch
    import torch.distributed as dist

    from . import _lib as L
    from .distributed import render_frame_adaptive
    from .scene import GlobalOpts, coordinate_system_debug, duration_debug_2, load_scene

    if "WORLD_SIZE" not in os.environ:  # plain `python -m`: a world of one
        os.environ.update({"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                           "MASTER_PORT": os.environ.get("MASTER_PORT", "29531")})
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n_dev = torch.cuda.device_count()
    if n_dev == 0:
        raise L.GrtError("no GPU visible: render_dist runs the HIP kernels only (there is no CPU path)")
    device = local_rank % n_dev
    torch.cuda.set_device(device)
    backend = a.backend or "nccl"
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", device))
    else:
        dist.init_process_group(backend)
    try:
        opts = GlobalOpts(width=a.width, height=a.height, step_size=a.step_size, max_steps=a.max_steps,
                          max_radius=a.max_radius, epsilon=a.epsilon, camera_position=a.camera_position, phi=a.phi,
                          theta=a.theta, psi=a.psi, tone_mapping=a.tone_mapping,
                          show_sampling_mask=a.show_sampling_mask, sampling_mask_color=a.sampling_mask_color)
        scene = load_scene(a.config_file, opts, a.resource_root)
        if rank == 0:
            hs = scene._keep  # main.rs:100-103, then the scene setup's lines (temperature.rs:55-102)
            _log(f"[render_dist] INFO Using coordinate system: {coordinate_system_debug(hs.desc.geometry, hs.desc.a)}")
            for line in hs.info_log:
                _log(f"[render_dist] INFO {line}")
            if a.filename.endswith(".hdr"):  # raytracer.rs:468-469, :481-483
                _log("[render_dist] INFO Creating HDR image")
            else:
                _log("[render_dist] INFO Creating non-HDR image")
                _log(f"[render_dist] INFO Tone mapping method: "
                     f"{ {'reinhard': 'Reinhard', 'global-linear': 'GlobalLinear'}[a.tone_mapping] }")
        mask = None
        if a.show_sampling_mask:
            mask = np.zeros(4)
            r, g, b = a.sampling_mask_color
            L.lib().grt_srgb_to_xyza(r, g, b, 255, L.dptr(mask))
        tone = {"reinhard": 0, "global-linear": 1}[a.tone_mapping]
        want_f64 = a.filename.endswith(".hdr") or a.raw_out is not None
        stats = torch.zeros(4, dtype=torch.int64, device=torch.device("cuda", device))
        dist.barrier()
        t0 = time.perf_counter()
        fail_cap = 1 << 20
        f_pix, f_smp, f_st = np.zeros(fail_cap, np.uint32), np.zeros(fail_cap, np.uint32), np.zeros(fail_cap, np.uint8)
        f_stop, f_steps = np.zeros(fail_cap, np.uint8), np.zeros(fail_cap, np.uint32)
        cfg = scene.adaptive
        supersampled = bool(cfg.enabled) or mask is not None
        if supersampled and rank == 0:  # raytracer.rs:264-267
            _log(f"[render_dist] INFO Rendering section from (0, 0) to ({scene.rows}, {scene.cols}) with supersampling")
        fails = None
        report = {}

        def render_once():
            nonlocal fails, report
            fails = L.SubsampleFailures(fail_cap, L.ptr(f_pix, C.c_uint32), L.ptr(f_smp, C.c_uint32),
                                        L.ptr(f_st, C.c_uint8), 0, L.ptr(f_stop, C.c_uint8), L.ptr(f_steps, C.c_uint32))
            report = {}
            stats.zero_()
            res = render_frame_adaptive(scene, rank, world, band_rows=a.band_rows, device=device, stats=stats,
                                        sampling_mask_xyza=mask, tone_mapping=None if want_f64 else tone,
                                        failures=C.byref(fails), report=report)
            torch.cuda.synchronize()
            return res

        def lost_pixels():
            # a device hit pool too small for some ray's candidates: every rank sees the sum
            lost = stats[3:4].clone() if dist.get_backend() != "gloo" else stats[3:4].cpu()
            dist.all_reduce(lost)
            return int(lost[0])

        def log_rank0(msg):
            if rank == 0:
                _log(f"[render_dist] {msg}")

        out, incomplete = trace_until_complete(
            render_once, lost_pixels,
            lambda: L.check(L.lib().grt_hit_pool_reserve(scene._s, device, 0, None), "grt_hit_pool_reserve"),
            log_rank0)
        t_render = time.perf_counter() - t0
        # each rank logs its own pixels, in pixel order (the reference logs from its parallel loop):
        # raytracer.rs:232-239 the failed pixels; scene.rs:178-183 / :196-202 the error-free rays that
        # ended on NaN coordinates or without a terminal event (steps.len() counts the initial step)
        st_local = report["status"].cpu().numpy().reshape(-1, scene.cols)
        stop_local = report["stop"].cpu().numpy().reshape(-1, scene.cols)
        steps_local = report["steps"].cpu().numpy().reshape(-1, scene.cols)
        for li, fi in zip(*np.nonzero((st_local & 0x7F) | np.isin(stop_local, (L.STOP_NAN, L.STOP_NONE)))):
            row = report["frame_rows"][li]
            if st_local[li, fi] & 0x7F:
                _log(f"[render_dist] ERROR Unable to compute color for ray at pixel ({fi}, {row}): "
                      f"{ERROR_NAMES.get(int(st_local[li, fi] & 0x7F), 'Unknown')}")
            else:
                log_ray_event(row, fi, int(stop_local[li, fi]), int(steps_local[li, fi]))
        if supersampled and mask is None:  # raytracer.rs:325 (rank 0: the frame's count), then the sub-rays
            if rank == 0:
                _log(f"[render_dist] INFO Supersampling {out[-1]} pixels")
            for k in range(min(int(fails.count), fail_cap)):
                row, col = divmod(int(f_pix[k]), scene.cols)
                if f_st[k]:
                    _log(f"[render_dist] ERROR Unable to compute color for ray at pixel ({col}, {row}): "
                          f"{ERROR_NAMES.get(int(f_st[k]), 'Unknown')}")
                else:
                    log_ray_event(row, col, int(f_stop[k]), int(f_steps[k]))
        if supersampled and rank == 0:  # raytracer.rs:313-316
            _log(f"[render_dist] INFO Finished rendering section from (0, 0) to ({scene.rows}, {scene.cols})")
        if dist.get_backend() == "gloo":
            host = stats.cpu()
            dist.all_reduce(host)
            totals = host
        else:
            dist.all_reduce(stats)
            totals = stats.cpu()
        if rank != 0:
            return exit_status(incomplete)
        w, h = scene.cols, scene.rows
        if want_f64:
            xyza64, _cls, _status, n_sel = out
            x = np.ascontiguousarray(xyza64.cpu().numpy())
            if a.raw_out is not None:
                x.tofile(a.raw_out)
            if a.filename.endswith(".hdr"):
                L.check(L.lib().grt_write_hdr_xyz(a.filename.encode(), L.dptr(x), w, h), "grt_write_hdr_xyz")
            else:
                rgb = np.zeros((w * h, 3), np.uint8)
                L.check(L.lib().grt_xyz_to_srgb8_device(device, L.dptr(x), w * h, tone, 1.0,
                                                        L.ptr(rgb, C.c_uint8)), "grt_xyz_to_srgb8_device")
                L.check(L.lib().grt_write_png_rgb(a.filename.encode(), L.ptr(rgb, C.c_uint8), w, h),
                        "grt_write_png_rgb")
        else:
            rgb_t, n_sel = out
            rgb = np.ascontiguousarray(rgb_t.cpu().numpy())
            L.check(L.lib().grt_write_png_rgb(a.filename.encode(), L.ptr(rgb, C.c_uint8), w, h), "grt_write_png_rgb")
        steps = int(totals[0])
        _log(f"[render_dist] {world} GPU(s): {int(totals[2])} rays, {steps} accepted steps, {int(totals[1])} attempts, "
              f"{n_sel} supersampled pixels, frame {t_render:.3f} s ({steps / t_render:.3e} steps/s)")
        _log(f"[render_dist] INFO saved image to {a.filename}")  # raytracer.rs:494, main.rs:175-176
        _log(f"[render_dist] INFO Elapsed time: {duration_debug_2(time.perf_counter() - t_start)}")
        return exit_status(incomplete)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
