"""C3 (1500^2 kerr-bl.toml) frames rendered RUNS times with the library in GRT_LIB:
md5 per run, and each run's per-pixel class / stop / steps / hits saved to OUT_<k>.npz
(the aee1fe7 nondeterminism study).  Usage: c3_det.py OUT [RUNS] [SAVE]"""
import hashlib
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

out = sys.argv[1]
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
save = int(sys.argv[3]) if len(sys.argv) > 3 else runs  # runs whose arrays are saved
opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-10.0, 0.0, -0.5), theta=-3.14159, max_steps=1000000)
hs = g.HostScene(str(ROOT / "tests/golden/scenes/kerr-bl.toml"), opts, str(ROOT / "tests/golden"))
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
for k in range(runs):
    r = sc.render_pixels(0, 0, 1500, 1500, aux=True)
    md5 = hashlib.md5(r.xyza.tobytes() + r.ray_class.tobytes()).hexdigest()[:12]
    if k < save:
        np.savez_compressed(f"{out}_{k}.npz", cls=r.ray_class, stop=r.stop_reason, steps=r.steps, hits=r.hits)
    print(json.dumps({"run": k, "md5": md5, "kernel_ms": r.stats["kernel_ms"], "accepted": r.stats["accepted_steps"],
                      "attempts": r.stats["attempts"]}), flush=True)
