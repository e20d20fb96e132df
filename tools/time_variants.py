"""Time the C2 (and C3) frame with each experimental libgrt build in variants/<name>/
(tools/build_variant.sh), one subprocess per variant and config, in the order given on
the command line (repeat names to alternate).  Frames must be identical (md5)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CODE = r'''
import sys, json, hashlib
sys.path.insert(0, "%s")
import gr_raytracer_amd as g
if "C3" in sys.argv:
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-10.0, 0.0, -0.5), theta=-3.14159, max_steps=1000000)
    hs = g.HostScene("%s/tests/golden/scenes/kerr-bl.toml", opts, "%s/tests/golden")
else:
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
    hs = g.HostScene("%s/tests/golden/scenes/schwarzschild.toml", opts, "%s/tests/golden")
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
ms = []
for i in range(3):
    r = sc.render_pixels(0, 0, 1500, 1500, aux=False)
    ms.append(r.stats["kernel_ms"])
st = r.stats
st["ms"] = ms
st["md5"] = hashlib.md5(r.xyza.tobytes() + r.ray_class.tobytes()).hexdigest()[:12]
print(json.dumps(st))
''' % ((ROOT,) * 5)
configs = os.environ.get("CONFIGS", "C2,C3").split(",")
for name in sys.argv[1:]:
    for cfg in configs:
        env = dict(os.environ, GRT_LIB=str(ROOT / "variants" / name / "libgrt.so"), GRT_LIB_ALLOW_MISSING="1")
        out = subprocess.run([sys.executable, "-c", CODE, cfg], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(name, "FAILED", out.stderr[-2000:], flush=True)
            sys.exit(1)
        st = json.loads(out.stdout.strip().splitlines()[-1])
        print(json.dumps({"variant": name, "config": cfg, "kernel_ms": [round(x, 1) for x in st["ms"]],
                          "accepted": st["accepted_steps"], "attempts": st["attempts"], "md5": st["md5"]}), flush=True)
