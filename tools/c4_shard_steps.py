"""Per-pixel accepted steps of one C4 row-band shard (tail analysis): writes
gpurun_out/<tag>/c4_shard<s>_steps.npy (local-row-major uint32)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g  # noqa: E402

tag, shard = sys.argv[1], int(sys.argv[2])
opts = g.GlobalOpts(width=4096, height=4096, camera_position=(-10.0, 0.0, -0.5), theta=1.52, psi=-1.57,
                    max_steps=1000000)
hs = g.HostScene(str(ROOT / "tests/golden/scenes/kerr.toml"), opts, str(ROOT / "tests/golden"))
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
r = sc.render_shard(16, shard, 8, aux=True)
out = ROOT / "gpurun_out" / tag
out.mkdir(parents=True, exist_ok=True)
np.save(out / f"c4_shard{shard}_steps.npy", r.steps)
np.save(out / f"c4_shard{shard}_stop.npy", r.stop_reason)
print(r.stats, flush=True)
