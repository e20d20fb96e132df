"""Kerr-Schild frames at the reference's example size (docs/example-render-commands.md:
1000x1000, camera -10,0,-0.5, theta 1.52, psi -1.57, max-steps 1e6): kerr.toml and the
volumetric kerr-volumetric-stony.toml, one timed frame each (after a small warm-up)."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import gr_raytracer_amd as g  # noqa: E402
from gr_raytracer_amd import _lib as L  # noqa: E402
from conftest import RESOURCES, SCENES, c4_opts  # noqa: E402

if "GRT_TAIL" in os.environ:
    L.check(L.lib().grt_set_tail(int(os.environ["GRT_TAIL"])))
size = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
for name in sys.argv[2:] or ["kerr.toml", "kerr-volumetric-stony.toml"]:
    hs = g.HostScene(str(SCENES / name), c4_opts(g, width=size, height=size), str(RESOURCES))
    sc = g.Scene(hs.desc_ptr(), keepalive=hs)
    sc.render_pixels(0, 0, 16, 16, aux=False)
    t0 = time.perf_counter()
    r = sc.render_pixels(aux=False)
    st = r.stats
    print(json.dumps({"scene": name, "pixels": size * size, "wall_s": round(time.perf_counter() - t0, 3),
                      "kernel_ms": st["kernel_ms"], "accepted_steps": st["accepted_steps"],
                      "march_jobs": st["march_jobs"], "march_samples": st["march_samples"],
                      "tail": os.environ.get("GRT_TAIL", "auto"), "handoffs": sc.tail_handoffs()}), flush=True)
