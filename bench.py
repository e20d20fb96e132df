"""bench.py — geodesic steps/sec/GPU on the reference's C2 configuration.

Workload (BASELINE.json configs[1]): 1500x1500 scene-definitions/schwarzschild.toml,
--max-steps=1e5, camera from README.md:63 (--camera-position=-16,0,3.5 --theta=-3.142),
1 sample per pixel (adaptive sampling off).  One bench "step" = one full 1500x1500
frame traced on the GPU (every pixel integrated to its stop condition, every window
tested against the Sphere and the Disc, every pixel shaded).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): weak
scaling over a batch of frames: rank r renders frame r of a camera fly-by (the camera
orbits the hole by r * 1e-3 rad), then the f32 frames are gathered to rank 0 over RCCL.
value = accepted steps of all ranks / max-over-ranks wall time.

Printed JSON carries the FP64 VALU roofline of the trace kernel (HIP events on the launch
stream) and the CPU baseline: the oracle (reference algorithm restated in C++, stored
trajectories + post-hoc window pass) timed on the host cores on a bounded row sample.
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

# algorithmic FP64 flops per accepted step = F_att * n_att + F_step
FLOPS = {  # geometry: (flops per RKF45 attempt, extra flops per accepted step)
    "schwarzschild": (733.0, 50.0),
    "kerr_bl": (865.0, 38.0),
    "kerr": (9913.0, 67.0),
}
FP64_VECTOR_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (AMD spec); see DESIGN.md
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md chip table
BYTES_PER_PIXEL_OUT = 16 + 1 + 1  # f32 XYZA + class + status


def c2_opts(g, frame: int = 0):
    ang = frame * 1e-3
    x, y, z = -16.0, 0.0, 3.5
    pos = (x * math.cos(ang) - y * math.sin(ang), x * math.sin(ang) + y * math.cos(ang), z)
    return g.GlobalOpts(width=1500, height=1500, camera_position=pos, theta=-3.142, psi=0.0, phi=0.0,
                        max_steps=100000)


def cpu_baseline(g, seconds_budget: float = 20.0) -> dict:
    """Oracle (reference algorithm) on rows = 0 mod 64 of the C2 frame, host cores."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle as O  # noqa: E402  (test infrastructure: the checker/baseline only)

    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))  # the GPU box's CPU share is 16
    hs = g.HostScene(str(ROOT / "tests/golden/scenes/schwarzschild.toml"), c2_opts(g),
                     str(ROOT / "tests/golden"))
    rows = list(range(0, 1500, 64))
    t0 = time.time()
    r = O.render_pixels(hs.desc, 0, 0, 1500, 1500, threads=cores, row_list=rows)
    wall = time.time() - t0
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": r["accepted"] / r["wall_s"], "unit": "geodesic steps/s", "cores": cores, "kind": "port",
            "cpu_model": model, "host_cpus": os.cpu_count(),
            "full_frame_s_extrapolated": round(r["wall_s"] * 1500 / len(rows), 1),
            "sample": f"C2 frame rows 0 mod 64 ({len(rows)} rows x 1500 px = {len(rows) * 1500} rays, "
                      f"{r['accepted']} accepted steps in {r['wall_s']:.1f} s, OpenMP dynamic over pixels)",
            "wall_s": round(wall, 2)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--blocks-per-cu", type=int, default=0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    else:
        torch.cuda.set_device(local_rank)
    dev = torch.device(f"cuda:{local_rank}")

    import gr_raytracer_amd as g
    from gr_raytracer_amd import _lib as L

    lib = L.lib()
    if args.blocks_per_cu:
        L.check(lib.grt_set_launch_config(args.blocks_per_cu, 256), "grt_set_launch_config")
    opts = c2_opts(g, frame=rank)
    hs = g.HostScene(str(ROOT / "tests/golden/scenes/schwarzschild.toml"), opts, str(ROOT / "tests/golden"))
    scene = g.Scene(hs.desc_ptr(), keepalive=hs)
    rows, cols = opts.height, opts.width
    n = rows * cols
    xyza = torch.empty((n, 4), dtype=torch.float32, device=dev)
    cls = torch.empty(n, dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    stats = torch.zeros(4, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    gather = [torch.empty_like(xyza) for _ in range(world)] if (world > 1 and rank == 0) else None

    def one_step():
        L.check(lib.grt_render_pixels_async(scene._s, local_rank, stream.cuda_stream, 0, 0, rows, cols,
                                            xyza.data_ptr(), cls.data_ptr(), status.data_ptr(), None, None, None,
                                            stats.data_ptr()), "grt_render_pixels_async")

    for _ in range(args.warmup):
        one_step()
        if world > 1:
            dist.gather(xyza, gather_list=gather, dst=0)
    torch.cuda.synchronize(dev)

    stats.zero_()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        one_step()
        ev[k][1].record(stream)
        if world > 1:
            dist.gather(xyza, gather_list=gather, dst=0)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    counters = stats.cpu().tolist()  # accepted, attempts, rays, overflows (summed over K frames)
    accepted, attempts = counters[0], counters[1]

    t = torch.tensor([elapsed, float(accepted), float(attempts)], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed = float(tmax[0])
    total_acc, total_att = float(t[1]), float(t[2])

    if rank == 0:
        f_att, f_step = FLOPS["schwarzschild"]
        acc_per_launch = accepted / args.steps
        att_per_launch = attempts / args.steps
        flop_per_launch = f_att * att_per_launch + f_step * acc_per_launch
        achieved_tflops = flop_per_launch / (kernel_ms * 1e-3) / 1e12
        prof = ROOT / "profiles" / "r01t_pmc.json"  # PMC passes of this kernel, tools/run_pmc.sh
        traffic = None
        if prof.exists():
            try:
                traffic = json.loads(prof.read_text()).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        line = {
            "metric": "geodesic steps/sec/GPU + wall-clock for 1500x1500 Schwarzschild render",
            "value": total_acc / elapsed,
            "unit": "accepted RKF45 geodesic steps/s (whole job)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: reference scene schwarzschild.toml + its textures (vendored fixtures)",
            "config": {"workload": "C2: 1500x1500 schwarzschild.toml, max-steps=1e5, camera -16,0,3.5 "
                                   "theta=-3.142, 1 spp (adaptive off); one step = one frame per GPU",
                       "frame_pixels": n, "parallelism": f"frames x{world} (one frame per GPU), RCCL gather",
                       "steps_per_gpu_per_s": total_acc / elapsed / world,
                       "attempts_per_accepted": total_att / max(total_acc, 1.0),
                       "frame_wall_s_per_gpu": elapsed / args.steps},
            "roofline": {"bound": "valu-fp64", "achieved": achieved_tflops, "peak": FP64_VECTOR_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved_tflops / FP64_VECTOR_PEAK_TFLOPS,
                         "traffic": traffic, "kernel": "grt::integrate_kernel<1, false> (Schwarzschild; events also span shade_kernel<1, 0>, <0.01%)",
                         "kernel_ms": kernel_ms, "flop_per_launch": flop_per_launch,
                         "flop_model": f"{f_att:g}*attempts + {f_step:g}*accepted (SURVEY 8d)",
                         "hbm_algorithmic_GBps": n * BYTES_PER_PIXEL_OUT / (kernel_ms * 1e-3) / 1e9,
                         "hbm_peak_GBps": HBM_PEAK_GBS},
            "cpu_baseline": None,
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(g)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
