"""Determinism / cross-build check of a full frame: render it twice with this build (and
once with GRT_REF_LIB's build in a subprocess), report differing pixels with their step
and hit counts.  python3 tools/diag_frames.py c3|c2"""
import json
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g  # noqa: E402

which = sys.argv[1]
if which == "c3":
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-10, 0, -0.5), theta=-3.14159, max_steps=1000000)
    toml = "kerr-bl.toml"
else:
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
    toml = "schwarzschild.toml"
hs = g.HostScene(str(ROOT / "tests/golden/scenes" / toml), opts, str(ROOT / "tests/golden"))
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
runs = [sc.render_pixels(0, 0, 1500, 1500) for _ in range(3)]
out = Path(sys.argv[2]) if len(sys.argv) > 2 else None
for k, r in enumerate(runs):
    print(json.dumps({"run": k, "accepted": r.stats["accepted_steps"], "kernel_ms": r.stats["kernel_ms"],
                      "hit_overflows": r.stats["hit_overflows"], "hits_max": int(r.hits.max()),
                      "rays_over_16_hits": int((r.hits > 16).sum()),
                      "flagged": int(((r.status & 0x80) != 0).sum())}), flush=True)
for k in (1, 2):
    d = np.flatnonzero(np.any(runs[k].xyza64 != runs[0].xyza64, axis=1) | (runs[k].steps != runs[0].steps))
    print(json.dumps({"run0_vs_run": k, "n_diff": int(d.size), "first": d[:10].tolist(),
                      "steps0": runs[0].steps[d[:10]].tolist(), "stepsk": runs[k].steps[d[:10]].tolist(),
                      "hits0": runs[0].hits[d[:10]].tolist()}), flush=True)
if out:
    np.savez_compressed(out, steps=runs[0].steps, hits=runs[0].hits, xyza=runs[0].xyza64, stop=runs[0].stop_reason,
                        status=runs[0].status)
