"""How many rhs<KERR> evaluations of a C4 row-band shard take the range-free metric
quotients (div_fx / sqrt_fx, ks_fd_ok true on every lane of the wave) and how many the
IEEE form.  Needs a diagnostic build (-DGRT_KS_PATH_COUNT=1, loaded through GRT_LIB):
counts are per wave (one lane counts each wave-level evaluation) and per lane.
Usage: tools/ks_path_count.py [N_SHARDS] [SHARD]"""
import ctypes as C
import hashlib
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g  # noqa: E402
from gr_raytracer_amd import _lib as L  # noqa: E402

n_shards = int(sys.argv[1]) if len(sys.argv) > 1 else 8
shard = int(sys.argv[2]) if len(sys.argv) > 2 else 2
opts = g.GlobalOpts(width=4096, height=4096, camera_position=(-10.0, 0.0, -0.5), theta=1.52, psi=-1.57,
                    max_steps=1000000)
hs = g.HostScene(str(ROOT / "tests/golden/scenes/kerr.toml"), opts, str(ROOT / "tests/golden"))
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
lib = L.lib()
fn = lib.grt_debug_ks_path
fn.restype = C.c_int
fn.argtypes = [C.POINTER(C.c_uint64), C.c_int]
cnt = (C.c_uint64 * 4)()
L.check(fn(cnt, 1), "grt_debug_ks_path")  # reset
t = time.time()
r = sc.render_shard(16, shard, n_shards, aux=False)
L.check(fn(cnt, 1), "grt_debug_ks_path")
w_fast, w_ieee, l_fast, l_ieee = (int(v) for v in cnt)
print(json.dumps({"shard": shard, "n_shards": n_shards, "wall_s": round(time.time() - t, 3),
                  "kernel_ms": r.stats["kernel_ms"], "attempts": r.stats["attempts"],
                  "wave_rhs_fast": w_fast, "wave_rhs_ieee": w_ieee, "lane_rhs_fast": l_fast, "lane_rhs_ieee": l_ieee,
                  "wave_fast_fraction": w_fast / max(1, w_fast + w_ieee),
                  "lane_fast_fraction": l_fast / max(1, l_fast + l_ieee),
                  "md5": hashlib.md5(r.xyza.tobytes() + r.ray_class.tobytes()).hexdigest()[:12]}), flush=True)
