"""C4 tail measurement: per-pixel steps of one 1/8 row-band shard (saved as .npy for
tools/tail_sim.py), then the longest ray of that shard traced alone (1x1 rectangle: one
lane on an otherwise idle GPU) and with its 8x8 tile (one full wave), timed, to give the
single-ray latency per accepted step that bounds the shard's makespan."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g  # noqa: E402

tag, shard = sys.argv[1], int(sys.argv[2])
out = ROOT / "gpurun_out" / tag
out.mkdir(parents=True, exist_ok=True)
opts = g.GlobalOpts(width=4096, height=4096, camera_position=(-10.0, 0.0, -0.5), theta=1.52, psi=-1.57,
                    max_steps=1000000)
hs = g.HostScene(str(ROOT / "tests/golden/scenes/kerr.toml"), opts, str(ROOT / "tests/golden"))
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
steps_file = out / f"c4_shard{shard}_steps.npy"
t = time.time()
r = sc.render_shard(16, shard, 8, aux=True)
print(json.dumps({"shard": shard, "wall_s": round(time.time() - t, 3), "kernel_ms": r.stats["kernel_ms"],
                  "accepted": r.stats["accepted_steps"]}), flush=True)
np.save(steps_file, r.steps)
steps = r.steps.reshape(-1, 4096)
lr, c = np.unravel_index(int(np.argmax(steps)), steps.shape)
fr = ((lr // 16) * 8 + shard) * 16 + lr % 16
for rect in [(fr, c, 1, 1), (fr - fr % 8, c - c % 8, 8, 8)]:
    t = time.time()
    p = sc.render_pixels(*rect)
    print(json.dumps({"rect": [int(v) for v in rect], "wall_s": round(time.time() - t, 3),
                      "kernel_ms": p.stats["kernel_ms"], "accepted": p.stats["accepted_steps"],
                      "attempts": p.stats["attempts"], "max_ray_steps": int(p.steps.max()),
                      "us_per_step_of_longest": p.stats["kernel_ms"] * 1e3 / max(int(p.steps.max()), 1)}), flush=True)
