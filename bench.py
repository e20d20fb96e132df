"""bench.py — geodesic steps/sec/GPU on the reference's C2 configuration.

Default workload (BASELINE.json configs[1]): 1500x1500 scene-definitions/schwarzschild.toml,
--max-steps=1e5, camera from README.md:63 (--camera-position=-16,0,3.5 --theta=-3.142),
1 sample per pixel (adaptive sampling off).  One bench "step" = one full 1500x1500
frame traced on the GPU (every pixel integrated to its stop condition, every window
tested against the Sphere and the Disc, every pixel shaded).  Two frames are in flight
(--inflight): frame k runs on slot k mod 2, each slot with its own Scene workspace, output
buffers and stream, so that one frame's end of pass overlaps the next frame's start; every
frame is traced in full, and the timed region ends when the last one is done.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): weak
scaling over a batch of frames: rank r renders frame r of a camera fly-by (the camera
orbits the hole by r * 1e-3 rad), then the f32 frames are gathered to rank 0 over RCCL.
value = accepted steps of all ranks / max-over-ranks wall time.

--workload c4 (BASELINE.json configs[3], the north-star layout): ONE 4096x4096 kerr.toml
frame (Kerr-Schild, max-steps 1e6, camera of docs/example-render-commands.md:29-37)
row-tiled across the N ranks (cyclic 16-row bands, grt_render_shard_async) and gathered
to rank 0 in one RCCL gather (gr_raytracer_amd.distributed.gather_frame).  Strong
scaling; the line carries each rank's kernel time, the max/mean imbalance and the
gather time.  A 4096^2 frame takes minutes per GPU: run it with --steps 1 --warmup 0.

Printed JSON carries the FP64 VALU roofline of the trace kernel (HIP events on the launch
stream) and the CPU baseline: the oracle (reference algorithm restated in C++, stored
trajectories + post-hoc window pass) timed on the host cores on a bounded sample.

The metric's second half, "wall-clock for 1500x1500 Schwarzschild render", is the
reference's own Elapsed time (main.rs:31, :175-176: CLI start -> image written): on one GPU
the C2 line also runs the `grt` CLI (the reference's `render` command line, README.md:63)
on the C2 scene at 1 spp and on the stock TOML (adaptive 4x4 supersampling, C5) and
reports the process wall time and the CLI's phase times (render_wall).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "geodesic steps/sec/GPU + wall-clock for 1500x1500 Schwarzschild render"
# algorithmic FP64 flops per accepted step = F_att * n_att + F_step
FLOPS = {  # geometry: (flops per RKF45 attempt, extra flops per accepted step)
    "schwarzschild": (733.0, 50.0),
    "kerr_bl": (865.0, 38.0),
    "kerr": (9913.0, 67.0),
}
FP64_VECTOR_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (AMD spec, FMA = 2 flops); see DESIGN.md
FP64_MEASURED_PEAK_TFLOPS = 61.8  # tools/fp64_peak.hip, profiles/r01/fp64_peak.json
# the path is compiled without contraction: every flop is one add / mul / div instruction
# slot, so the issue ceiling for this arithmetic is half the FMA peak
FP64_NO_CONTRACTION_TFLOPS = FP64_VECTOR_PEAK_TFLOPS / 2
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md chip table
BYTES_PER_PIXEL_OUT = 16 + 1 + 1  # f32 XYZA + class + status
# the kernel whose PMC summary (profiles/*_pmc.json, tools/pmc_summary.py) gives `traffic`
PMC_DIR = ROOT / "profiles"
PMC_KERNEL = {"c2": "grt::integrate_kernel<1, false>", "c4": "grt::integrate_kernel<2, false>"}
SCENES = ROOT / "tests" / "golden" / "scenes"


def c2_opts(g, frame: int = 0):
    ang = frame * 1e-3
    x, y, z = -16.0, 0.0, 3.5
    pos = (x * math.cos(ang) - y * math.sin(ang), x * math.sin(ang) + y * math.cos(ang), z)
    return g.GlobalOpts(width=1500, height=1500, camera_position=pos, theta=-3.142, psi=0.0, phi=0.0,
                        max_steps=100000)


def c4_opts(g, size: int = 4096, max_steps: int = 1000000):
    return g.GlobalOpts(width=size, height=size, camera_position=(-10.0, 0.0, -0.5), theta=1.52, psi=-1.57,
                        phi=0.0, max_steps=max_steps)


# ----------------------------------------------------------------- host cores ----
def host_cores() -> dict:
    """The CPUs this process may use: its affinity set, the cgroup CPU quota (the GPU
    box's lease), physical cores and SMT among them."""
    try:
        aff = sorted(os.sched_getaffinity(0))
    except Exception:
        aff = list(range(os.cpu_count() or 1))
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        if q != "max":
            quota = float(q) / float(period)
    except Exception:
        pass
    phys = set()
    model = ""
    try:
        cpu = core = pkg = None
        for ln in Path("/proc/cpuinfo").read_text().splitlines():
            if ln.startswith("processor"):
                cpu = int(ln.split(":")[1])
            elif ln.startswith("physical id"):
                pkg = ln.split(":")[1].strip()
            elif ln.startswith("core id"):
                core = ln.split(":")[1].strip()
            elif ln.startswith("model name") and not model:
                model = ln.split(":", 1)[1].strip()
            elif not ln.strip() and cpu is not None:
                if cpu in aff:
                    phys.add((pkg, core))
                cpu = core = pkg = None
    except Exception:
        pass
    smt = None
    try:
        smt = Path("/sys/devices/system/cpu/smt/active").read_text().strip() == "1"
    except Exception:
        pass
    threads = len(aff)
    if quota is not None:  # more runnable threads than the quota only adds throttling
        threads = max(1, min(threads, int(math.ceil(quota))))
    return {"threads": threads, "affinity_cpus": len(aff), "cgroup_cpu_quota": quota,
            "physical_cores_in_affinity": len(phys) or None, "smt_active": smt, "cpu_model": model,
            "host_cpus": os.cpu_count()}


def cpu_baseline(g, workload: str = "c2") -> dict:
    """The oracle (reference algorithm, kind "port") on a bounded sample of the same
    workload, on every host core this process may use (affinity set, capped only by the
    cgroup quota when one is set)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import numpy as np
    import pyoracle as O  # noqa: E402  (test infrastructure: the checker/baseline only)

    hc = host_cores()
    cores = hc["threads"]
    if workload == "c4":
        hs = g.HostScene(str(SCENES / "kerr.toml"), c4_opts(g), str(ROOT / "tests/golden"))
        rng = np.random.default_rng(13)
        cell = 128
        r0, c0 = np.meshgrid(np.arange(0, 4096, cell), np.arange(0, 4096, cell), indexing="ij")
        ri = (r0.ravel() + rng.random(r0.size) * cell).astype(np.int64)
        ci = (c0.ravel() + rng.random(c0.size) * cell).astype(np.int64)
        pix = (ri * 4096 + ci).astype(np.uint32)
        half = np.full(pix.size, 0.5)
        t0 = time.time()
        r = O.render_pixels(hs.desc, 0, 0, 4096, 4096, threads=cores, offsets=(pix, half, half))
        wall = time.time() - t0
        sample = (f"C4 frame, 1024 stratified pixels (one per 128x128 cell, pixel centre), {r['accepted']} accepted "
                  f"steps in {r['wall_s']:.1f} s, OpenMP dynamic over pixels")
        extra = {}
    else:
        hs = g.HostScene(str(SCENES / "schwarzschild.toml"), c2_opts(g), str(ROOT / "tests/golden"))
        stride = 16 if cores >= 64 else 64  # rows = 0 mod 16 on a large host
        rows = list(range(0, 1500, stride))
        t0 = time.time()
        r = O.render_pixels(hs.desc, 0, 0, 1500, 1500, threads=cores, row_list=rows)
        wall = time.time() - t0
        sample = (f"C2 frame rows 0 mod {stride} ({len(rows)} rows x 1500 px = {len(rows) * 1500} rays, "
                  f"{r['accepted']} accepted steps in {r['wall_s']:.1f} s, OpenMP dynamic over pixels)")
        extra = {"full_frame_s_extrapolated": round(r["wall_s"] * 1500 / len(rows), 1)}
    out = {"value": r["accepted"] / r["wall_s"], "unit": "geodesic steps/s", "cores": cores, "kind": "port",
           "sample": sample, "wall_s": round(wall, 2)}
    out.update(extra)
    out.update({k: v for k, v in hc.items() if k != "threads"})
    return out


# ------------------------------------------------------------------- roofline ----
def find_pmc(workload: str, rays: int):
    """The newest PMC summary under profiles/ that measured THIS build's code of the
    workload's integrate kernel (kernel_code_sha256, or the whole device code's hash for
    summaries that predate it) on a launch of `rays` rays (per-launch traffic is only
    comparable between launches of the same size).  Returns (path, summary, note)."""
    from gr_raytracer_amd import _lib as L

    kname = PMC_KERNEL[workload]
    mine_k = L.kernel_code_sha256(L.kernel_symbol(kname))
    mine_all = L.device_code_sha256()
    stale, other_size = [], []
    for prof in sorted(PMC_DIR.glob("*_pmc.json"), reverse=True):
        try:
            pmc = json.loads(prof.read_text())
        except ValueError:
            continue
        if not pmc.get("kernel", "").startswith(kname + ","):
            continue
        if pmc.get("kernel_code_sha256") == mine_k or pmc.get("code_object_sha256") == mine_all:
            if pmc.get("rays_per_launch") == rays:
                return prof, pmc, None
            other_size.append(prof.name)
            continue
        stale.append(prof.name)
    if other_size:
        return None, None, (f"PMC summaries of this build's {kname} ({', '.join(other_size[:3])}) measured launches "
                            f"of another size than {rays} rays: not used")
    if stale:
        return None, None, f"PMC summaries of {kname} ({', '.join(stale[:3])}) measured another build: not used"
    return None, None, f"no PMC summary of {kname}"


def roofline(workload: str, geometry: str, accepted: float, attempts: float, kernel_ms: float,
             n_pixels: int, kernel_name: str) -> dict:
    """FP64 VALU roofline of the integrate kernel for one launch (counts per launch)."""
    from gr_raytracer_amd import _lib as L

    f_att, f_step = FLOPS[geometry]
    flop = f_att * attempts + f_step * accepted
    achieved = flop / (kernel_ms * 1e-3) / 1e12
    out = {"bound": "valu-fp64", "achieved": achieved, "peak": FP64_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
           "frac": achieved / FP64_VECTOR_PEAK_TFLOPS,
           "frac_measured_peak": achieved / FP64_MEASURED_PEAK_TFLOPS,
           "frac_no_contraction": achieved / FP64_NO_CONTRACTION_TFLOPS,
           "traffic": None, "kernel": kernel_name, "kernel_ms": kernel_ms, "flop_per_launch": flop,
           "flop_model": f"{f_att:g}*attempts + {f_step:g}*accepted (SURVEY 8d)",
           "hbm_algorithmic_GBps": n_pixels * BYTES_PER_PIXEL_OUT / (kernel_ms * 1e-3) / 1e9,
           "hbm_peak_GBps": HBM_PEAK_GBS}
    prof, pmc, note = find_pmc(workload, n_pixels)
    if pmc is None:
        out["traffic_note"] = note
    else:
        out["traffic"] = pmc.get("hbm_bytes_per_launch")
        out["pmc_file"] = os.path.relpath(prof, ROOT)
        for k in ("active_valu_over_wave_cycles", "lane_utilisation", "valu_f64_fraction",
                  "wait_inst_any_over_wave_cycles", "scratch_bytes_per_launch"):
            if k in pmc:
                out[k] = pmc[k]
    return out


# ------------------------------------------------------------------ workloads ----
def reduce_over_ranks(elapsed: float, accepted: float, attempts: float, world: int, device="cpu"):
    """The weak-scaling line's job totals: the max over ranks of the timed region and the
    sums of every rank's accepted steps and attempts (backend-agnostic: RCCL on the GPUs,
    gloo in tests)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([elapsed, float(accepted), float(attempts)], dtype=torch.float64, device=device)
    if world > 1:
        tmax = t[:1].clone()
        steps = t[1:].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(steps, op=dist.ReduceOp.SUM)
        return float(tmax[0]), float(steps[0]), float(steps[1])
    return float(t[0]), float(t[1]), float(t[2])


# ---------------------------------------------------------------- CLI wall ----
README_FLAGS = ["--width=1500", "--height=1500", "--camera-position=-16.0,0.0,3.5", "--theta=-3.142", "--psi=0.0",
                "--phi=0.0", "--max-steps=100000"]  # README.md:63, BASELINE configs[1]


def parse_cli_phases(stderr: str) -> dict:
    """The `[grt] phases (ms): load L, create C, render R, output O, write W, since start S`
    line and the reference's `Elapsed time: ...` line of a `grt ... render` run."""
    import re

    out = {}
    m = re.search(r"\[grt\] phases \(ms\): (.*)", stderr)
    if m:
        for part in m.group(1).split(","):
            k, v = part.strip().rsplit(" ", 1)
            out[k.replace(" ", "_") + "_ms"] = float(v)
    m = re.search(r"INFO Elapsed time: (\S+)", stderr)
    if m:
        out["elapsed_line"] = m.group(1)
    m = re.search(r"\[grt\] (\d+) rays, (\d+) accepted steps", stderr)
    if m:
        out["rays"], out["accepted_steps"] = int(m.group(1)), int(m.group(2))
    return out


def cli_wall(adaptive: bool, device: int = 0, reps: int = 2) -> dict:
    """`grt ... render` on the C2 scene (BASELINE's wall-clock half): process start -> exit
    with the PNG written, best of `reps` runs (each a fresh process: HIP runtime start, TOML
    and texture decode, upload, trace, tone map, PNG encode).  adaptive=False renders the
    1-spp C2 frame (the TOML with [adaptive_sampling] enabled = false, the fixture BASELINE.md
    names); True the stock TOML, whose default adaptive 4x4 supersampling makes it C5."""
    import subprocess
    import tempfile

    exe = ROOT / "gr_raytracer_amd" / "lib" / "grt"
    with tempfile.TemporaryDirectory() as d:
        toml = SCENES / "schwarzschild.toml"
        if not adaptive:
            toml = Path(d) / "schwarzschild-1spp.toml"
            toml.write_text((SCENES / "schwarzschild.toml").read_text() + "\n[adaptive_sampling]\nenabled = false\n")
        png = Path(d) / "render.png"
        runs = []
        for _ in range(reps):
            if png.exists():
                png.unlink()
            cmd = [str(exe), *README_FLAGS, "--device", str(device), "--resource-root", str(ROOT / "tests/golden"),
                   "--config-file", str(toml), "render", "--filename", str(png)]
            t0 = time.perf_counter()
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            wall = time.perf_counter() - t0
            if r.returncode != 0 or not png.exists():
                return {"error": f"grt exited {r.returncode}: {r.stderr[-400:]}"}
            runs.append((wall, parse_cli_phases(r.stderr)))
    wall, phases = min(runs, key=lambda x: x[0])
    return {"render_wall_s": round(wall, 3), "runs_s": [round(w, 3) for w, _ in runs],
            "command": "grt " + " ".join(README_FLAGS) + f" --config-file {toml.name} render",
            "scene": "schwarzschild.toml" + ("" if adaptive else " + [adaptive_sampling] enabled = false (1 spp)"),
            "phases": phases}


def c2_frame_loop(n_slots: int, steps: int, warmup: int, render, gather, sync, barrier, reset, record=None) -> float:
    """The C2 weak-scaling loop, backend-agnostic (RCCL streams on the GPUs, gloo in tests).
    Frame k goes to slot k mod n_slots: render(slot) enqueues it, gather(slot) (or None)
    sends it to rank 0, record(k, 0 | 1, slot) brackets the render for the device events.
    A warm-up step renders one frame in every slot; reset() then clears the counters.
    Returns the timed region's wall time (barrier and sync on both sides)."""
    for _ in range(warmup):
        for j in range(n_slots):
            render(j)
            if gather is not None:
                gather(j)
    sync()
    reset()
    barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        j = k % n_slots
        if record is not None:
            record(k, 0, j)
        render(j)
        if record is not None:
            record(k, 1, j)
        if gather is not None:
            gather(j)
    sync()
    barrier()
    return time.perf_counter() - t0


def run_c2(args, rank, world, local_rank, dev):
    import torch
    import torch.distributed as dist

    import gr_raytracer_amd as g
    from gr_raytracer_amd import _lib as L

    lib = L.lib()
    opts = c2_opts(g, frame=rank)
    hs = g.HostScene(str(SCENES / "schwarzschild.toml"), opts, str(ROOT / "tests/golden"))
    rows, cols = opts.height, opts.width
    n = rows * cols
    # Frames in flight: frame k goes to slot k mod F, each slot with its own Scene (device
    # workspace, counters), output buffers and stream, so that the persistent kernel's end of
    # pass (the last ray lifetime at falling lane occupancy) overlaps the next frame's start.
    F = max(1, args.inflight)
    gathered = world > 1 or args.self_gather  # --self-gather: the gather path in a group of one
    slots = []
    for _ in range(F):
        slots.append({
            "scene": g.Scene(hs.desc_ptr(), keepalive=hs),
            "xyza": torch.empty((n, 4), dtype=torch.float32, device=dev),
            "cls": torch.empty(n, dtype=torch.uint8, device=dev),
            "status": torch.empty(n, dtype=torch.uint8, device=dev),
            "stats": torch.zeros(4, dtype=torch.int64, device=dev),
            "stream": torch.cuda.current_stream(dev) if F == 1 else torch.cuda.Stream(dev),
            "gather": [torch.empty((n, 4), dtype=torch.float32, device=dev) for _ in range(world)]
            if (gathered and rank == 0) else None,
        })

    def render(j):
        s = slots[j]
        L.check(lib.grt_render_pixels_async(s["scene"]._s, local_rank, s["stream"].cuda_stream, 0, 0, rows, cols,
                                            s["xyza"].data_ptr(), s["cls"].data_ptr(), s["status"].data_ptr(),
                                            None, None, None, s["stats"].data_ptr()), "grt_render_pixels_async")

    def gather(j):  # on the slot's stream: the gather waits for this frame only, and the
        s = slots[j]  # slot's next frame waits for the gather
        with torch.cuda.stream(s["stream"]):
            dist.gather(s["xyza"], gather_list=s["gather"], dst=0, async_op=True).wait()

    def reset():
        for s in slots:
            s["stats"].zero_()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    elapsed = c2_frame_loop(F, args.steps, args.warmup, render, gather if gathered else None,
                            lambda: torch.cuda.synchronize(dev), (lambda: dist.barrier()) if world > 1 else (lambda: None),
                            reset, lambda k, e, j: ev[k][e].record(slots[j]["stream"]))
    # the device time per frame: first frame's start to last frame's end over K (with one
    # frame in flight, the mean launch duration)
    if F == 1:
        kernel_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    else:  # the last frame to finish is one of the last F
        kernel_ms = max(ev[0][0].elapsed_time(e[1]) for e in ev[-F:]) / args.steps
    counters = [sum(v) for v in zip(*(s["stats"].cpu().tolist() for s in slots))]
    accepted, attempts = counters[0], counters[1]  # summed over K frames
    # One frame alone in flight (after the timed region, untimed): a single launch's own
    # duration, the basis of frac_single_launch beside the pipelined throughput fraction.
    single_ms = []
    if args.single_launches > 0:
        s0 = slots[0]
        for _ in range(args.single_launches):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0["stats"].zero_()
            torch.cuda.synchronize(dev)
            e0.record(s0["stream"])
            render(0)
            e1.record(s0["stream"])
            e1.synchronize()
            single_ms.append(e0.elapsed_time(e1))
        single_counts = s0["stats"].cpu().tolist()

    elapsed, total_acc, total_att = reduce_over_ranks(elapsed, accepted, attempts, world, dev)
    if rank != 0:
        return None
    line = {
        "metric": METRIC,
        "value": total_acc / elapsed,
        "unit": "accepted RKF45 geodesic steps/s (whole job)",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: reference scene schwarzschild.toml + its textures (vendored fixtures)",
        "config": {"workload": "C2: 1500x1500 schwarzschild.toml, max-steps=1e5, camera -16,0,3.5 "
                               "theta=-3.142, 1 spp (adaptive off); one step = one frame per GPU",
                   "frame_pixels": n, "parallelism": f"frames x{world} (one frame per GPU), RCCL gather",
                   "frames_in_flight": F,
                   "steps_per_gpu_per_s": total_acc / elapsed / world,
                   "attempts_per_accepted": total_att / max(total_acc, 1.0),
                   "accepted_steps_per_frame": total_acc / (args.steps * world),
                   # wall time per frame of the timed loop (with F frames in flight: the
                   # throughput period, not one frame's latency; see single_launch_ms)
                   "frame_period_s": elapsed / args.steps},
        "roofline": roofline("c2", "schwarzschild", accepted / args.steps, attempts / args.steps, kernel_ms, n,
                             "grt::integrate_kernel<1, false> (Schwarzschild; events also span shade_kernel<1, 0>, "
                             "<0.01%)"),
        "cpu_baseline": None,
    }
    # each timed frame's own span between its two events on its slot's stream (with frames in
    # flight a span includes the time the frame shares the CUs with its neighbours)
    line["roofline"]["frame_event_ms"] = [round(a.elapsed_time(b), 1) for a, b in ev]
    line["roofline"]["kernel_ms_basis"] = (
        "mean launch duration (HIP events on the launch stream)" if F == 1 else
        f"pipelined throughput: device time per frame with {F} frames in flight, first frame's start event to "
        f"last frame's end event / K (HIP events on the slots' streams); a single launch's duration overlaps its "
        f"neighbours' (rocprof: the spacing of consecutive integrate-kernel ends, tools/kernel_period.py), so this "
        f"frac is a throughput fraction; frac_single_launch is one launch's")
    if single_ms:
        r1 = roofline("c2", "schwarzschild", single_counts[0], single_counts[1], min(single_ms), n, "")
        line["roofline"]["single_launch_ms"] = [round(v, 2) for v in single_ms]
        line["roofline"]["frac_single_launch"] = r1["frac"]
        line["roofline"]["single_launch_basis"] = (
            f"{len(single_ms)} frames rendered alone after the timed region (one in flight, slot 0's stream), "
            f"shortest launch; HIP events around grt_render_pixels_async (integrate + shade kernels)")
    if world == 1 and args.fused_check and args.arith == "exact":
        # the same loop in the fused arithmetic mode (grt_set_arithmetic(1): FMA contraction in
        # the light charts' kernels, pixels within 1e-4 of the reference on every robust pixel,
        # tests/test_fused.py), measured beside the exact headline
        g.set_arithmetic("fused")
        try:
            evf = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.steps)]
            el_f = c2_frame_loop(F, args.steps, 1, render, None, lambda: torch.cuda.synchronize(dev),
                                 lambda: None, reset, lambda k, e, j: evf[k][e].record(slots[j]["stream"]))
            kms_f = (sum(a.elapsed_time(b) for a, b in evf) / args.steps if F == 1 else
                     max(evf[0][0].elapsed_time(e[1]) for e in evf[-F:]) / args.steps)
            cf = [sum(v) for v in zip(*(s["stats"].cpu().tolist() for s in slots))]
        finally:
            g.set_arithmetic("exact")
        rf = roofline("c2", "schwarzschild", cf[0] / args.steps, cf[1] / args.steps, kms_f, n, "")
        line["fused"] = {"value": cf[0] / el_f, "ms_per_step": el_f / args.steps * 1e3, "kernel_ms": kms_f,
                         "frac": rf["frac"], "accepted_steps_per_frame": cf[0] / args.steps,
                         "speedup_vs_exact": (elapsed / args.steps) / (el_f / args.steps),
                         "mode": "grt_set_arithmetic(1): the light charts' kernels with FMA contraction "
                                 "(geodesic_fused.hip); same loop, frames and slots as the headline; parity bar "
                                 "1e-4 relative per channel on every robust pixel (tests/test_fused.py), not bit "
                                 "identity"}
    if world == 1 and not args.no_cli_wall:
        torch.cuda.synchronize(dev)
        line["render_wall"] = {"c2_1spp": cli_wall(False, local_rank), "c5_adaptive": cli_wall(True, local_rank)}
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline(g, "c2")
    return line


def c4_frame_steps(trace_shard, rank: int, world: int, frame_rows: int, cols: int, band_rows: int,
                   steps: int, warmup: int, sync, group=None):
    """The C4 strong-scaling loop, backend-agnostic (RCCL on the GPUs, gloo in tests).

    trace_shard() traces this rank's row bands and returns (records (n_local, 18) u8,
    accepted, attempts, kernel_ms); sync() waits for the rank's device.  Per step:
    barrier, trace, barrier (every rank's kernel done), ONE gather of the records to
    rank 0.  Returns this rank's per-step lists and the frames' accepted/attempt sums."""
    import torch.distributed as dist

    from gr_raytracer_amd.distributed import gather_frame

    for _ in range(warmup):
        rec, _, _, _ = trace_shard()
        gather_frame(rec, frame_rows, cols, band_rows, rank, world, 0, group)
    sync()
    kernel_ms, gather_ms, step_s = [], [], []
    acc = att = 0.0
    frame = None
    for _ in range(steps):
        dist.barrier(group=group)
        sync()
        t0 = time.perf_counter()
        rec, a, b, kms = trace_shard()
        sync()
        acc += a
        att += b
        kernel_ms.append(kms)
        dist.barrier(group=group)  # every rank's shard is traced
        t1 = time.perf_counter()
        frame = gather_frame(rec, frame_rows, cols, band_rows, rank, world, 0, group)
        sync()
        t2 = time.perf_counter()
        gather_ms.append((t2 - t1) * 1e3)
        step_s.append(t2 - t0)
    return {"kernel_ms": kernel_ms, "gather_ms": gather_ms, "step_s": step_s, "accepted": acc, "attempts": att,
            "frame": frame}


def c4_summary(res: dict, rank: int, world: int, device="cpu", group=None) -> dict:
    """Reduce c4_frame_steps' per-rank results: max-over-ranks step time, per-rank
    kernel ms, imbalance = max / mean kernel ms, gather ms on rank 0."""
    import torch
    import torch.distributed as dist

    steps = len(res["step_s"])
    mine = torch.tensor([sum(res["step_s"]), sum(res["kernel_ms"]) / steps, res["accepted"], res["attempts"]],
                        dtype=torch.float64, device=device)
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine, group=group)
    allv = [v.cpu() for v in allv]
    if rank != 0:
        return None
    per_rank_ms = [float(v[1]) for v in allv]
    elapsed = max(float(v[0]) for v in allv)
    mean_ms = sum(per_rank_ms) / world
    return {"elapsed_s": elapsed, "per_rank_kernel_ms": per_rank_ms,
            "imbalance": max(per_rank_ms) / mean_ms if mean_ms > 0 else 1.0,
            "gather_ms": sum(res["gather_ms"]) / steps,
            "accepted": sum(float(v[2]) for v in allv), "attempts": sum(float(v[3]) for v in allv),
            "rank0_accepted": float(allv[0][2]), "rank0_attempts": float(allv[0][3]), "steps": steps}


def run_c4(args, rank, world, local_rank, dev):
    import ctypes as C

    import torch
    import torch.distributed as dist

    import gr_raytracer_amd as g
    from gr_raytracer_amd import _lib as L
    from gr_raytracer_amd.distributed import pack_records, shard_row_count

    lib = L.lib()
    opts = c4_opts(g, args.size)
    hs = g.HostScene(str(SCENES / "kerr.toml"), opts, str(ROOT / "tests/golden"))
    scene = g.Scene(hs.desc_ptr(), keepalive=hs)
    rows, cols, band = opts.height, opts.width, args.band_rows
    n_local = shard_row_count(rows, band, rank, world) * cols
    xyza = torch.empty((n_local, 4), dtype=torch.float32, device=dev)
    cls = torch.empty(n_local, dtype=torch.uint8, device=dev)
    status = torch.empty(n_local, dtype=torch.uint8, device=dev)
    stats = torch.zeros(4, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = L.RowShard(band, rank, world)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def trace_shard():
        stats.zero_()
        e0.record(stream)
        L.check(lib.grt_render_shard_async(scene._s, local_rank, stream.cuda_stream, C.byref(sh), xyza.data_ptr(),
                                           cls.data_ptr(), status.data_ptr(), None, None, None, stats.data_ptr()),
                "grt_render_shard_async")
        e1.record(stream)
        e1.synchronize()
        c = stats.cpu().tolist()
        return pack_records(xyza, cls, status), float(c[0]), float(c[1]), e0.elapsed_time(e1)

    res = c4_frame_steps(trace_shard, rank, world, rows, cols, band, args.steps, args.warmup,
                         lambda: torch.cuda.synchronize(dev))
    s = c4_summary(res, rank, world, dev)
    if rank != 0:
        return None
    line = {
        "metric": METRIC,
        "value": s["accepted"] / s["elapsed_s"],
        "unit": "accepted RKF45 geodesic steps/s (whole job)",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": s["elapsed_s"] / s["steps"] * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: reference scene kerr.toml + its textures (vendored fixtures)",
        "config": {"workload": f"C4: {cols}x{rows} kerr.toml (Kerr-Schild), max-steps=1e6, camera -10,0,-0.5 "
                               "theta=1.52 psi=-1.57, 1 spp; one step = one frame row-tiled across the ranks",
                   "frame_pixels": rows * cols, "band_rows": band,
                   "parallelism": f"cyclic {band}-row bands x{world}, one RCCL gather to rank 0",
                   "steps_per_gpu_per_s": s["accepted"] / s["elapsed_s"] / world,
                   "attempts_per_accepted": s["attempts"] / max(s["accepted"], 1.0),
                   "frame_wall_s": s["elapsed_s"] / s["steps"]},
        "per_rank_kernel_ms": s["per_rank_kernel_ms"],
        "imbalance": s["imbalance"],
        "gather_ms": s["gather_ms"],
        "gather_GBps": rows * cols * BYTES_PER_PIXEL_OUT / (s["gather_ms"] * 1e-3) / 1e9 if s["gather_ms"] else None,
        "roofline": roofline("c4", "kerr", s["rank0_accepted"] / s["steps"], s["rank0_attempts"] / s["steps"],
                             s["per_rank_kernel_ms"][0], n_local, "grt::integrate_kernel<2, false> + grt::tail_kernel<2, false> "
                             "(Kerr-Schild; the events also span the probe pass and shade_kernel<2, 0>; "
                             "traffic: the integrate kernel's PMC summary only), rank 0's shard"),
        "cpu_baseline": None,
    }
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline(g, "c4")
    return line


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed frames (default: c2 6, c4 1); the first two frames in flight start together and "
                    "overlap more than later ones (DESIGN.md section 6), so more frames weigh that start less")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=("c2", "c4"), default="c2")
    ap.add_argument("--size", type=int, default=4096, help="c4: frame edge (4096 = configs[3])")
    ap.add_argument("--band-rows", type=int, default=16, help="c4: rows per cyclic band")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inflight", type=int, default=2,
                    help="c2: frames in flight (one stream and workspace each); 1 = one frame after another")
    ap.add_argument("--blocks-per-cu", type=int, default=0)
    ap.add_argument("--single-launches", type=int, default=2,
                    help="c2: frames rendered alone after the timed region (frac_single_launch)")
    ap.add_argument("--no-cli-wall", action="store_true", help="c2: skip the grt CLI wall-clock runs")
    ap.add_argument("--arith", choices=("exact", "fused"), default="exact",
                    help="grt_set_arithmetic for the timed loop (exact: the reference's roundings)")
    ap.add_argument("--no-fused-check", dest="fused_check", action="store_false",
                    help="c2, one GPU: skip the extra fused-mode measurement")
    ap.add_argument("--self-gather", action="store_true", help="c2, one GPU: run the multi-GPU gather path "
                    "in a process group of one (a check of the streams and RCCL gathers)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 6 if args.workload == "c2" else 1

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    elif args.workload == "c4" or args.self_gather:  # barriers / the gather path: a group of one
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(f"cuda:{local_rank}"))
    dev = torch.device(f"cuda:{local_rank}")

    from gr_raytracer_amd import _lib as L

    if args.blocks_per_cu:
        L.check(L.lib().grt_set_launch_config(args.blocks_per_cu, 256), "grt_set_launch_config")
    L.check(L.lib().grt_set_arithmetic(1 if args.arith == "fused" else 0), "grt_set_arithmetic")
    line = (run_c4 if args.workload == "c4" else run_c2)(args, rank, world, local_rank, dev)
    if line is not None:
        line["source_hash"] = L.source_stamp()  # the sources libgrt.so was built from (checked on load)
        line["arith"] = args.arith
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
