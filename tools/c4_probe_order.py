"""Probe keys and tile queue order of one C4 1/8 row-band shard (band 16), from a diagnostic
build (GRT_LIB=variants/rt/libgrt.so, -DGRT_RAY_TIMES=1): writes OUT.npz (probe, order).

usage: python tools/c4_probe_order.py OUT.npz [SHARD=2] [N_SHARDS=8]"""
import ctypes as C
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
sh = L.RowShard(16, shard, n_shards)
rows = int(L.lib().grt_shard_row_count(4096, C.byref(sh)))
n = (rows // 8) * 512
probe, order = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
f = L.lib().grt_debug_probe_order
f.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
L.check(f(sc._s, 0, C.byref(sh), probe.ctypes.data, order.ctypes.data, n), "grt_debug_probe_order")
np.savez_compressed(out, probe=probe, order=order)
print(n, int(probe.max()), int((probe > 20000).sum()), order[:10].tolist(), flush=True)
