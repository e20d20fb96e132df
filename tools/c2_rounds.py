"""C2 kernel time against the frame height: the rays are uniform (~15.5k steps), so a
frame takes ceil(rays / lanes) rounds of one ray per lane; time per ray shows the cost
of a partly filled last round.  Heights chosen for 14.0 .. 17.17 rays per lane (rows from the top of the frame)."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g  # noqa: E402

lanes = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
hs = g.HostScene(str(ROOT / "tests/golden/scenes/schwarzschild.toml"), opts, str(ROOT / "tests/golden"))
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
sc.render_pixels(0, 0, 1500, 1500, aux=False)  # warm-up
for per_lane in (14.0, 14.5, 15.0, 15.5, 16.0, 16.5, 17.0, 17.17):
    rows = min(1500, int(per_lane * lanes / 1500))
    r = sc.render_pixels(0, 0, rows, 1500, aux=False)
    st = r.stats
    print(json.dumps({"rows": rows, "rays": rows * 1500, "rays_per_lane": rows * 1500 / lanes,
                      "kernel_ms": st["kernel_ms"], "accepted": st["accepted_steps"],
                      "ns_per_step": st["kernel_ms"] * 1e6 / st["accepted_steps"]}), flush=True)
