"""Profiling target: one C2 frame (c2), one C3 frame (c3), the C4 1/8 row-band shard 2
(c4: 4096^2 kerr.toml, band 16, the north-star layout's rank 2) or the whole C4 frame in
one launch (c4full: bench.py --workload c4 on one GPU).
python3 tools/prof_target.py [c2|c3|c4|c4full]"""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g
import os
if "GRT_SCHEDULE" in os.environ:  # -1 auto, 0 row-major tiles, 1 probe-ordered
    g.lib().grt_set_schedule(int(os.environ["GRT_SCHEDULE"]))
which = sys.argv[1] if len(sys.argv) > 1 else "c2"
if which == "c2":
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
    toml = "schwarzschild.toml"
elif which in ("c4", "c4full"):
    opts = g.GlobalOpts(width=4096, height=4096, camera_position=(-10.0, 0.0, -0.5), theta=1.52, psi=-1.57,
                        max_steps=1000000)
    toml = "kerr.toml"
else:
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-10, 0, -0.5), theta=-3.14159, max_steps=1000000)
    toml = "kerr-bl.toml"
hs = g.HostScene(str(ROOT / "tests/golden/scenes" / toml), opts, str(ROOT / "tests/golden"))
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
if which == "c4":
    r = sc.render_shard(16, 2, 8, aux=False)
elif which == "c4full":
    r = sc.render_shard(16, 0, 1, aux=False)
else:
    r = sc.render_pixels(0, 0, opts.height, opts.width, aux=False)
print(r.stats)
