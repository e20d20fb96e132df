"""C2 frame kernel time under each tile-queue order (grt_set_schedule 0: row-major 8x8
tiles, 1: probe-ordered longest-first), alternating; frames must be identical."""
import hashlib
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g  # noqa: E402
from gr_raytracer_amd import _lib as L  # noqa: E402

opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
hs = g.HostScene(str(ROOT / "tests/golden/scenes/schwarzschild.toml"), opts, str(ROOT / "tests/golden"))
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
w = sc.render_pixels(0, 0, 1500, 1500, aux=True)  # warm-up, and the per-pixel step counts
import numpy as np  # noqa: E402
st = w.steps.astype(np.int64)
print(json.dumps({"steps_percentiles": {q: int(np.percentile(st, q)) for q in (1, 10, 50, 90, 99, 100)},
                  "mean": float(st.mean()), "share_of_steps_in_rays_below_5000": float(st[st < 5000].sum() / st.sum()),
                  "last_64_rows_mean": float(st.reshape(1500, 1500)[-64:].mean())}), flush=True)
for mode in [int(m) for m in (sys.argv[1:] or ["0", "1", "0", "1"])]:
    L.check(L.lib().grt_set_schedule(mode))
    r = sc.render_pixels(0, 0, 1500, 1500, aux=False)
    print(json.dumps({"schedule": mode, "kernel_ms": r.stats["kernel_ms"], "accepted": r.stats["accepted_steps"],
                      "md5": hashlib.md5(r.xyza.tobytes() + r.ray_class.tobytes()).hexdigest()[:12]}), flush=True)
L.lib().grt_set_schedule(-1)
