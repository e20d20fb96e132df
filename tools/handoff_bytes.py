"""The integrate -> shade hand-off of one launch, from the windows-with-hits count of
every ray (RenderResult.hits, scene.rs:141-152): per-ray records (64-B final state +
16-B meta), candidate records in workspace slots (64 B each, the first GRT_MAX_HITS = 16
of a ray) and hit-pool records beyond them (~65 B: window, object, momentum, point, link).
These are the bytes the integrate kernel must write; the PMC WRITE_SIZE of the same
launch (tools/run_pmc.sh) minus them is scratch (spills) and queue / counter traffic.

python3 tools/handoff_bytes.py [c2|c3|c4|c4full]   (c4 = shard 2 of 8, band 16, as prof_target;
c4full = the whole 4096^2 frame in one launch)"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g  # noqa: E402

SLOTS, REC, POOL = 16, 64, 65
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
# ray record: 64 B (KerrBL: 64 B + its 16-B meta record)
RAY = 80 if which == "c3" else 64
if which == "c4":
    r = sc.render_shard(16, 2, 8)
elif which == "c4full":
    r = sc.render_shard(16, 0, 1)
else:
    r = sc.render_pixels(0, 0, opts.height, opts.width)
hits = r.hits.astype(np.int64)
n = len(hits)
slots = int(np.minimum(hits, SLOTS).sum())
pool = int(np.maximum(hits - SLOTS, 0).sum())
out = {"config": which, "rays": n, "windows_with_hits": int(hits.sum()), "rays_with_hits": int((hits > 0).sum()),
       "max_hits": int(hits.max()), "slot_records": slots, "pool_records": pool,
       "ray_record_bytes": RAY * n, "slot_record_bytes": REC * slots, "pool_record_bytes": POOL * pool,
       "handoff_bytes": RAY * n + REC * slots + POOL * pool, "kernel_ms": r.stats["kernel_ms"]}
print(json.dumps(out))
