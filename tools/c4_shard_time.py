"""C4 (4096^2 kerr.toml, Kerr-Schild) on one GPU: time the row-band shards an 8-GPU
node would give each rank (band 16), to size the multi-GPU C4 run."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import gr_raytracer_amd as g  # noqa: E402

opts = g.GlobalOpts(width=4096, height=4096, camera_position=(-10.0, 0.0, -0.5), theta=1.52, psi=-1.57,
                    max_steps=1000000)
hs = g.HostScene(str(ROOT / "tests/golden/scenes/kerr.toml"), opts, str(ROOT / "tests/golden"))
sc = g.Scene(hs.desc_ptr(), keepalive=hs)
import os  # noqa: E402
from gr_raytracer_amd import _lib as L  # noqa: E402
if "GRT_SCHEDULE" in os.environ:  # -1 auto, 0 row-major tiles, 1 probe-ordered
    L.check(L.lib().grt_set_schedule(int(os.environ["GRT_SCHEDULE"])))
if "GRT_TWO_ENDED" in os.environ:  # 1 (default) both ends of the tile queue, 0 one end
    L.check(L.lib().grt_set_two_ended(int(os.environ["GRT_TWO_ENDED"])))
if "GRT_TAIL" in os.environ:  # -1 auto, 0 off, > 0 hand-off threshold
    L.check(L.lib().grt_set_tail(int(os.environ["GRT_TAIL"])))
import hashlib  # noqa: E402
n_shards = int(sys.argv[1]) if len(sys.argv) > 1 else 8
shards = [int(x) for x in sys.argv[2:]] or [0, n_shards // 2]
for s in shards:
    t = time.time()
    r = sc.render_shard(16, s, n_shards, aux=True)
    st = r.stats
    rep = sc.tail_report(capacity=1 << 20)
    tail = {k: round(rep[k], 3) for k in ("drained_s", "handoff_s", "tail_end_s")}
    if rep["handed_off"]:
        rem = r.steps.astype("int64")[rep["slot"].astype("int64")] - rep["step"].astype("int64")
        tail.update(max_remaining=int(rem.max()), mean_remaining=float(rem.mean()),
                    longest_at_handoff=int(rep["step"][int(rem.argmax())]),
                    us_per_step_tail=round((rep["tail_end_s"] - rep["handoff_s"]) * 1e6 / max(int(rem.max()), 1), 2))
    print(json.dumps({"shard": s, "n_shards": n_shards, "rays": st["rays"], "wall_s": round(time.time() - t, 3),
                      "kernel_ms": st["kernel_ms"], "accepted": st["accepted_steps"], "attempts": st["attempts"],
                      "steps_per_s": st["accepted_steps"] / (st["kernel_ms"] * 1e-3),
                      "overflows": st["hit_overflows"], "schedule": os.environ.get("GRT_SCHEDULE", "auto"),
                      "tail": os.environ.get("GRT_TAIL", "auto"),
                      "two_ended": os.environ.get("GRT_TWO_ENDED", "1"), "handoffs": sc.tail_handoffs(), "tail_timeline": tail,
                      "md5": hashlib.md5(r.xyza.tobytes() + r.ray_class.tobytes()).hexdigest()[:12]}), flush=True)
