import sys, time, json
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT) + "")
import gr_raytracer_amd as g
from gr_raytracer_amd import _lib as L
opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
hs = g.HostScene(str(ROOT) + "/tests/golden/scenes/schwarzschild.toml", opts, str(ROOT) + "/tests/golden")
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
for bpc, thr in [(4, 256), (2, 256), (8, 128), (16, 64), (4, 256), (2, 256)]:
    L.check(L.lib().grt_set_launch_config(bpc, thr))
    r = sc.render_pixels(0, 0, 1500, 1500, aux=False)
    print(json.dumps({"bpc": bpc, "threads": thr, "kernel_ms": r.stats["kernel_ms"]}), flush=True)
