"""Profiling target for the device output stage (output.hip): a 4096 x 4096 f64 XYZA
framebuffer (C4's size, 537 MB, synthetic HDR values) mapped 5 times per tone mapping
on torch's stream.  Reports the HBM rate from HIP events; rocprofv3 gives the per-kernel
durations.  python3 tools/prof_output.py"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gr_raytracer_amd import _lib as L  # noqa: E402

lib = L.lib()
n = 4096 * 4096
g = torch.Generator(device="cuda").manual_seed(7)
x = torch.rand((n, 4), dtype=torch.float64, device="cuda", generator=g) * 3.0
m = torch.zeros(3, dtype=torch.float64, device="cuda")
rgb = torch.empty((n, 3), dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream()
out = {}
for tone in (0, 1):
    for k in range(6):  # first iteration is the warm-up
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(s)
        if tone == 1:
            L.check(lib.grt_linear_max_async(0, s.cuda_stream, x.data_ptr(), n, 1.0, m.data_ptr()))
        e1.record(s)
        L.check(lib.grt_tonemap_async(0, s.cuda_stream, x.data_ptr(), n, tone, 1.0, m.data_ptr(), rgb.data_ptr()))
        e2.record(s)
        torch.cuda.synchronize()
        if k:
            out.setdefault(tone, []).append((e0.elapsed_time(e1), e1.elapsed_time(e2)))
res = {}
for tone, v in out.items():
    mx = sum(a for a, _ in v) / len(v)
    tm = sum(b for _, b in v) / len(v)
    res["reinhard" if tone == 0 else "global_linear"] = {
        "max_ms": mx, "tonemap_ms": tm,
        "tonemap_GBps": n * (32 + 3) / (tm * 1e-3) / 1e9,
        "max_GBps": (n * 32 / (mx * 1e-3) / 1e9) if mx > 0.001 else None}
print(json.dumps({"pixels": n, "algorithmic_bytes_per_pixel": {"tonemap": 35, "linear_max": 32}, **res}))
