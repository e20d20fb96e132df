"""Early hand-off diagnostics on a C4 crop (max-steps 1e5): stats and per-ray sums with the
hand-off off / on, plus the early report (debugging aid)."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g  # noqa: E402

opts = g.GlobalOpts(width=4096, height=4096, camera_position=(-10.0, 0.0, -0.5), theta=1.52, psi=-1.57,
                    max_steps=100000)
hs = g.HostScene(str(ROOT / "tests/golden/scenes/kerr.toml"), opts, str(ROOT / "tests/golden"))
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
rect = (1816, 2792, 24, 24)
for steps, cus in ((0, 0), (1, 8), (1, 8), (5000, 32)):
    g.scene.set_early_tail(steps, cus)
    r = sc.render_pixels(*rect)
    print(json.dumps({"early": [steps, cus], "stats": {k: r.stats[k] for k in ("accepted_steps", "attempts", "rays")},
                      "sum_steps": int(r.steps.astype(np.int64).sum()), "report": sc.early_report(),
                      "handoffs": sc.tail_handoffs()}), flush=True)
