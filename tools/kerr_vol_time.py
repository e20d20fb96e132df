"""Kerr-Schild frames at the reference's example size (docs/example-render-commands.md:
1000x1000, camera -10,0,-0.5, theta 1.52, psi -1.57, max-steps 1e6): kerr.toml and the
volumetric kerr-volumetric-stony.toml, one timed frame each (after a small warm-up), with
the long-ray hand-off timeline and the step-count tail of the frame."""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

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
    r = sc.render_pixels(aux=True)
    wall = time.perf_counter() - t0
    st = r.stats
    rep = sc.tail_report(capacity=1 << 20)
    tl = {k: round(rep[k], 3) for k in ("drained_s", "handoff_s", "tail_end_s")}
    steps = r.steps.astype(np.int64)
    if rep["handed_off"]:
        rem = steps[rep["slot"].astype(np.int64)] - rep["step"].astype(np.int64)
        tl.update(max_remaining=int(rem.max()), longest_at_handoff=int(rep["step"][int(rem.argmax())]))
        # the ray that ends last: its tile's probe key as schedule.hip forms it (pixel (3, 3)
        # of each 8x8 tile, capped at 1.3 max_radius, max over the 3x3 tile neighbourhood)
        crit = int(rep["slot"][int(rem.argmax())])
        cr, cc = divmod(crit, size)
        tiles_y, tiles_x = (size + 7) // 8, (size + 7) // 8
        grid = steps.reshape(size, size)
        cap = int(min(max(1.3 * 15000.0, 4096), 32768))
        probe = np.zeros((tiles_y, tiles_x), np.int64)
        for ty in range(tiles_y):
            for tx in range(tiles_x):
                r, c = ty * 8 + 3, tx * 8 + 3
                probe[ty, tx] = min(int(grid[r, c]), cap) if r < size and c < size else 0
        pad = np.pad(probe, 1)
        key = np.max([pad[1 + dy:1 + dy + tiles_y, 1 + dx:1 + dx + tiles_x] for dy in (-1, 0, 1) for dx in (-1, 0, 1)],
                     axis=0)
        k = key[cr // 8, cc // 8]
        tl.update(critical_pixel=[cr, cc], critical_steps=int(grid[cr, cc]), critical_tile_key=int(k),
                  tiles_with_higher_key=int((key > k).sum()), tiles_at_cap=int((key >= cap).sum()),
                  tiles=int(tiles_x * tiles_y))
    print(json.dumps({"scene": name, "pixels": size * size, "wall_s": round(wall, 3), "kernel_ms": st["kernel_ms"],
                      "accepted_steps": st["accepted_steps"], "march_jobs": st["march_jobs"],
                      "march_samples": st["march_samples"], "tail": os.environ.get("GRT_TAIL", "auto"),
                      "handoffs": int(rep["handed_off"]), "timeline": tl,
                      "rays_over": {str(k): int((steps > k).sum()) for k in (100000, 300000, 500000, 900000)},
                      "max_steps_rays": int((steps >= 999999).sum())}), flush=True)
