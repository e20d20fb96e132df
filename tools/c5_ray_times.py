"""Per-ray schedule of C5's supersample pass (the sub-ray trace of grt_render_section) from
a diagnostic build (tools/build_variant.sh rt 's/x/x/' -DGRT_RAY_TIMES=1, loaded through
GRT_LIB): each sub-ray's start and end (s since its integrate kernel started), attempts
and accepted steps, and the live-ray count over time (the ramp-down of a pass of ~2.5
rays per lane).  usage: python tools/c5_ray_times.py OUT.npz"""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g  # noqa: E402
from gr_raytracer_amd import _lib as L  # noqa: E402

out = sys.argv[1]
opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
hs = g.HostScene(str(ROOT / "tests/golden/scenes/schwarzschild.toml"), opts, str(ROOT / "tests/golden"))
ad = hs.adaptive
ad.enabled = 1
sc = g.Scene(hs.desc_ptr(), keepalive=hs, adaptive=ad)
only = L.lib().grt_debug_ray_times_only
only.argtypes = [C.c_uint64]
L.check(only(2), "grt_debug_ray_times_only")  # trace 1: the 1-spp frame, trace 2: the sub-ray chunk
_, _, n_sel, st = sc.render_section()
f = L.lib().grt_debug_ray_times
f.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(C.c_uint64)]
n = 1 << 21  # the supersample chunk (api.hip SUB_CHUNK): the last trace's slots
buf = np.zeros(6 * n, np.uint64)
t0 = C.c_uint64()
L.check(f(sc._s, 0, buf.ctypes.data_as(C.POINTER(C.c_uint64)), n, C.byref(t0)), "grt_debug_ray_times")
w = buf.reshape(6, n)
live = w[0] > 0
t_first = np.int64(w[0][live].min())  # the kernel's first ray start (t0 is kept only by Kerr-Schild)
start = ((w[0][live].astype(np.int64) - t_first) * 1e-8).astype(np.float32)
end = ((w[2][live].astype(np.int64) - t_first) * 1e-8).astype(np.float32)
att = w[4][live].astype(np.uint32)
np.savez_compressed(out, start=start, end=end, att=att)
t_end = float(end.max())
grid = np.linspace(0.0, t_end, 201)
active = [(int(((start <= t) & (end > t)).sum())) for t in grid]
lanes = 196608  # 256 CUs x 4 SIMDs x 3 waves x 64 lanes (integrate_waves(1) = 3)
busy = np.trapezoid(active, grid) / (lanes * t_end)
print(json.dumps({"selected": n_sel, "sub_rays": int(live.sum()), "kernel_end_s": t_end,
                  "last_start_s": float(start.max()), "mean_ray_s": float((end - start).mean()),
                  "lane_occupancy": float(busy), "attempts": int(att.sum()),
                  "active_at": {f"{t:.4f}": a for t, a in zip(grid[::10], active[::10])},
                  "section_kernel_ms": st["kernel_ms"]}), flush=True)
