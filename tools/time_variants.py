"""Time the C2 frame with each experimental libgrt variant (one subprocess each)."""
import json, os, subprocess, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
CODE = r'''
import sys, time, json
sys.path.insert(0, "%s")
import gr_raytracer_amd as g
if "C3" in sys.argv:
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-10.0, 0.0, -0.5), theta=-3.14159, max_steps=1000000)
    hs = g.HostScene("%s/tests/golden/scenes/kerr-bl.toml", opts, "%s/tests/golden")
else:
    opts = g.GlobalOpts(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
    hs = g.HostScene("%s/tests/golden/scenes/schwarzschild.toml", opts, "%s/tests/golden")
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
best = None
for i in range(2):
    r = sc.render_pixels(0, 0, 1500, 1500, aux=False)
    st = r.stats
    if best is None or st["kernel_ms"] < best["kernel_ms"]:
        best = st
import hashlib
best["md5"] = hashlib.md5(r.xyza.tobytes()).hexdigest()[:12]
print(json.dumps(best))
''' % ((ROOT,) * 5)
for name in sys.argv[1:]:
  for cfg in ("C2", "C3"):
    env = dict(os.environ, GRT_LIB=str(ROOT / "variants" / name / "libgrt.so"), GRT_LIB_ALLOW_MISSING="1")
    out = subprocess.run([sys.executable, "-c", CODE, cfg], env=env, capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        print(name, "FAILED", out.stderr[-2000:], flush=True)
        sys.exit(1)
    st = json.loads(out.stdout.strip().splitlines()[-1])
    print(f"{name:16s} {cfg} kernel {st['kernel_ms']:9.1f} ms  steps/s {st['accepted_steps']/st['kernel_ms']*1e3:.3e} "
          f"attempts {st['attempts']} frame-md5 {st['md5']}", flush=True)
