"""C5 (BASELINE configs[4]): 1500x1500 schwarzschild.toml with the stock TOML's adaptive
4x4 supersampling (render_section_to_cie_buffer_supersampled, raytracer.rs:246-458),
fully on the GPU via grt_render_section.  Prints wall time, selected pixels, steps."""
import hashlib
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g  # noqa: E402
import os  # noqa: E402
if "GRT_BLOCKS_PER_CU" in os.environ:  # integrate-kernel blocks per CU (default: 2 x waves per SIMD)
    g._lib.check(g._lib.lib().grt_set_launch_config(int(os.environ["GRT_BLOCKS_PER_CU"]), 256), "grt_set_launch_config")

opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
hs = g.HostScene(str(ROOT / "tests/golden/scenes/schwarzschild.toml"), opts, str(ROOT / "tests/golden"))
ad = hs.adaptive
ad.enabled = 1  # the stock TOMLs supersample by default
sc = g.Scene(hs.desc_ptr(), keepalive=hs, adaptive=ad)
for k in range(2):
    t = time.time()
    out, cls, n_sel, st = sc.render_section()
    wall = time.time() - t
    print(json.dumps({"run": k, "wall_s": round(wall, 3), "kernel_ms": st["kernel_ms"], "supersampled_pixels": n_sel,
                      "rays": st["rays"], "accepted_steps": st["accepted_steps"],
                      "md5": hashlib.md5(out.tobytes()).hexdigest()[:12],
                      "steps_per_s": st["accepted_steps"] / wall,
                      "adaptive": {"samples_per_axis": ad.samples_per_axis,
                                   "luminance_contrast_threshold": ad.luminance_contrast_threshold}}), flush=True)
