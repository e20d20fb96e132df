"""Code-path counts of the integrate kernel on one workload, from a diagnostic build
(-DGRT_PATH_COUNT=1, loaded through GRT_LIB; geodesic.hip path_count): per path, how many
times a wave executed it (counted by its first active lane) and how many lanes did.
Kerr-Schild RHS: 0 range-free, 1 IEEE.  Schwarzschild / KerrBL RHS: 0 region-B table
with range-free divisions, 1 region-B Taylor with them, 2 region B with IEEE divisions,
3 general sincos (7: of those, with the range-free divisions).  All: 4 near-field window pass, 5 accepted step, 6 attempt.
usage: tools/path_count.py c2|c3|c4 (c4: row-band shard 2 of 8)"""
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

which = sys.argv[1] if len(sys.argv) > 1 else "c2"
if which == "c4":
    opts = g.GlobalOpts(width=4096, height=4096, camera_position=(-10.0, 0.0, -0.5), theta=1.52, psi=-1.57,
                        max_steps=1000000)
    toml = "kerr.toml"
elif which == "c3":
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-10.0, 0.0, -0.5), theta=-3.14159, max_steps=1000000)
    toml = "kerr-bl.toml"
else:
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
    toml = "schwarzschild.toml"
hs = g.HostScene(str(ROOT / "tests/golden/scenes" / toml), opts, str(ROOT / "tests/golden"))
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
fn = L.lib().grt_debug_path_counts
fn.restype = C.c_int
fn.argtypes = [C.POINTER(C.c_uint64), C.c_int]
cnt = (C.c_uint64 * 16)()
L.check(fn(cnt, 1), "grt_debug_path_counts")  # reset
t = time.time()
r = sc.render_shard(16, 2, 8, aux=False) if which == "c4" else sc.render_pixels(0, 0, 1500, 1500, aux=False)
L.check(fn(cnt, 1), "grt_debug_path_counts")
names = (["rhs_range_free", "rhs_ieee"] if which == "c4" else
         ["rhs_b_table_fast", "rhs_b_taylor_fast", "rhs_b_ieee", "rhs_general"]) 
names += ["near_window", "accepted_general_path", "attempt"]
keys = [0, 1] if which == "c4" else [0, 1, 2, 3]
keys += [4, 5, 6]
if which != "c4":  # general sincos with the range-free divisions (GRT_FAST_DIV_GEN builds)
    names.append("rhs_general_range_free")
    keys.append(7)
out = {"workload": which, "kernel_ms": r.stats["kernel_ms"], "wall_s": round(time.time() - t, 3),
       "accepted_steps": r.stats["accepted_steps"], "attempts_total": r.stats["attempts"],
       "md5": hashlib.md5(r.xyza.tobytes() + r.ray_class.tobytes()).hexdigest()[:12]}
for nm, k in zip(names, keys):
    w, ln = int(cnt[k]), int(cnt[8 + k])
    out[nm] = {"waves": w, "lanes": ln, "lanes_per_wave": round(ln / w, 2) if w else 0.0}
print(json.dumps(out), flush=True)
