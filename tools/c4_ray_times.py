"""Per-ray schedule of one C4 1/8 row-band shard (band 16) on one GPU, from a diagnostic
build (tools/build_variant.sh rt 's/x/x/' -DGRT_RAY_TIMES=1; GRT_LIB=variants/rt/libgrt.so):
for every ray its start, hand-off and end time (s since the integrate kernel started),
the hardware place of the lane that started it (XCC, SE, CU, SIMD, wave slot), its
attempts in the integrate and tail kernels and its accepted steps.  Writes a compressed
.npz (tools/c4_sched_sim.py calibrates its model against it).

usage: python tools/c4_ray_times.py OUT.npz [SHARD=2] [N_SHARDS=8]"""
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
shard = int(sys.argv[2]) if len(sys.argv) > 2 else 2
n_shards = int(sys.argv[3]) if len(sys.argv) > 3 else 8
opts = g.GlobalOpts(width=4096, height=4096, camera_position=(-10.0, 0.0, -0.5), theta=1.52, psi=-1.57,
                    max_steps=1000000)
hs = g.HostScene(str(ROOT / "tests/golden/scenes/kerr.toml"), opts, str(ROOT / "tests/golden"))
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
r = sc.render_shard(16, shard, n_shards, aux=True)
n = r.steps.size
buf = np.zeros(6 * n, np.uint64)
t0 = C.c_uint64()
f = L.lib().grt_debug_ray_times
f.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(C.c_uint64)]
L.check(f(sc._s, 0, buf.ctypes.data_as(C.POINTER(C.c_uint64)), n, C.byref(t0)), "grt_debug_ray_times")
w = buf.reshape(6, n)


def sec(v):
    return np.where(v > 0, (v.astype(np.int64) - np.int64(t0.value)) * 1e-8, -1.0).astype(np.float32)


hw = (w[3] & 0xffffffff).astype(np.uint32)
xcc = (w[3] >> 32).astype(np.uint32)
# gfx9 HW_ID: wave [3:0], SIMD [5:4], CU [11:8], SH [12], SE [15:13]
place = ((xcc & 7) << 16) | (((hw >> 13) & 7) << 13) | (((hw >> 12) & 1) << 12) | (((hw >> 8) & 15) << 8) | \
        (((hw >> 4) & 3) << 4) | (hw & 15)
np.savez_compressed(out, start=sec(w[0]), handoff=sec(w[1]), end=sec(w[2]), place=place.astype(np.uint32),
                    att_int=w[4].astype(np.uint32), att_tail=w[5].astype(np.uint32),
                    steps=r.steps.astype(np.uint32), stop=r.stop_reason.astype(np.uint8))
rep = sc.tail_report()
print(json.dumps({"shard": shard, "rays": int(n), "kernel_ms": r.stats["kernel_ms"],
                  "accepted": r.stats["accepted_steps"], "attempts": r.stats["attempts"],
                  "drained_s": rep["drained_s"], "handoff_s": rep["handoff_s"], "tail_end_s": rep["tail_end_s"],
                  "end_max_s": float(sec(w[2]).max()), "places": int(np.unique(place).size)}), flush=True)
