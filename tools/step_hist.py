"""Per-ray step-count distribution of a workload (C2 frame or a C4 row-band shard):
python3 tools/step_hist.py c2|c4 [n_shards shard] -> summary line + gpurun_out/steps_<tag>.npy"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g  # noqa: E402

which = sys.argv[1]
if which == "c2":
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
    toml = "schwarzschild.toml"
elif which == "c3":
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-10, 0, -0.5), theta=-3.14159, max_steps=1000000)
    toml = "kerr-bl.toml"
else:
    opts = g.GlobalOpts(width=4096, height=4096, camera_position=(-10.0, 0.0, -0.5), theta=1.52, psi=-1.57,
                        max_steps=1000000)
    toml = "kerr.toml"
hs = g.HostScene(str(ROOT / "tests/golden/scenes" / toml), opts, str(ROOT / "tests/golden"))
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
if which == "c4":
    n_shards, shard = int(sys.argv[2]), int(sys.argv[3])
    r = sc.render_shard(16, shard, n_shards)
    tag = f"c4_{n_shards}_{shard}"
else:
    r = sc.render_pixels(0, 0, opts.height, opts.width)
    tag = which
s = r.steps.astype(np.int64)
out = ROOT / "gpurun_out"
out.mkdir(exist_ok=True)
np.save(out / f"steps_{tag}.npy", r.steps)
np.save(out / f"stop_{tag}.npy", r.stop_reason)
q = np.percentile(s, [50, 90, 99, 99.9, 99.99, 100]).tolist()
print(json.dumps({"tag": tag, "rays": int(s.size), "total": int(s.sum()), "kernel_ms": r.stats["kernel_ms"],
                  "pct_50_90_99_999_9999_max": q, "n_ge_1e5": int((s >= 100000).sum()),
                  "n_ge_5e5": int((s >= 500000).sum()), "stop_counts": np.bincount(r.stop_reason).tolist(),
                  "status_counts": np.bincount(r.status).tolist()}), flush=True)
