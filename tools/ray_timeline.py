"""Per-ray schedule of one integrate launch from a diagnostic build (tools/build_variant.sh
rt 's/x/x/' -DGRT_RAY_TIMES=1, loaded through GRT_LIB): C2's whole frame (c2), C3's (c3:
kerr-bl.toml, the C3 camera) or C5's supersample pass (c5: trace 2 of grt_render_section).  Prints the live-ray count over
time, the time the queue drained (last ray start), the kernel's end and the lane
occupancy (live-ray time over lanes x span); saves start / end / attempts to OUT.npz.
usage: python tools/ray_timeline.py c2|c3|c5 OUT.npz"""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g  # noqa: E402
import os  # noqa: E402
if "GRT_BLOCKS_PER_CU" in os.environ:  # integrate-kernel blocks per CU (default: 2 x waves per SIMD)
    g._lib.check(g._lib.lib().grt_set_launch_config(int(os.environ["GRT_BLOCKS_PER_CU"]), 256), "grt_set_launch_config")
from gr_raytracer_amd import _lib as L  # noqa: E402

mode, out = sys.argv[1], sys.argv[2]
if mode == "c3":
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-10.0, 0.0, -0.5), theta=-3.14159, max_steps=1000000)
    hs = g.HostScene(str(ROOT / "tests/golden/scenes/kerr-bl.toml"), opts, str(ROOT / "tests/golden"))
else:
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
    hs = g.HostScene(str(ROOT / "tests/golden/scenes/schwarzschild.toml"), opts, str(ROOT / "tests/golden"))
lib = L.lib()
only = lib.grt_debug_ray_times_only
only.argtypes = [C.c_uint64]
if mode == "c5":
    ad = hs.adaptive
    ad.enabled = 1
    sc = g.Scene(hs.desc_ptr(), keepalive=hs, adaptive=ad)
    L.check(only(2), "grt_debug_ray_times_only")  # trace 1: the 1-spp frame, trace 2: the sub-ray chunk
    sc.render_section()
    n = 1 << 21  # the supersample chunk's slots (api.hip SUB_CHUNK)
else:
    sc = g.Scene(hs.desc_ptr(), keepalive=hs)
    L.check(only(0), "grt_debug_ray_times_only")
    sc.render_pixels(0, 0, 1500, 1500, aux=False)
    n = 1500 * 1500
f = lib.grt_debug_ray_times
f.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(C.c_uint64)]
buf = np.zeros(6 * n, np.uint64)
t0 = C.c_uint64()
L.check(f(sc._s, 0, buf.ctypes.data_as(C.POINTER(C.c_uint64)), n, C.byref(t0)), "grt_debug_ray_times")
w = buf.reshape(6, n)
live = w[0] > 0
t_first = np.int64(w[0][live].min())
start = (w[0][live].astype(np.int64) - t_first) * 1e-8
end = (w[2][live].astype(np.int64) - t_first) * 1e-8
att = w[4][live].astype(np.uint32)
np.savez_compressed(out, start=start.astype(np.float32), end=end.astype(np.float32), att=att)
t_end = float(end.max())
grid = np.linspace(0.0, t_end, 401)
order_s, order_e = np.sort(start), np.sort(end)
active = np.searchsorted(order_s, grid, "right") - np.searchsorted(order_e, grid, "right")
lanes = 196608  # 256 CUs x 4 SIMDs x 3 waves x 64 lanes (integrate_waves(1) = 3)
busy = float(np.trapezoid(active, grid) / (lanes * t_end))
t_drain = float(start.max())
print(json.dumps({"mode": mode, "rays": int(live.sum()), "kernel_end_s": t_end, "last_start_s": t_drain,
                  "after_drain_s": t_end - t_drain, "mean_ray_s": float((end - start).mean()), "lane_occupancy": busy,
                  "live_at": {f"{t:.3f}": int(a) for t, a in zip(grid[::20], active[::20])}}), flush=True)
