"""C2 frames back to back on one stream against frames alternating over two streams, each
stream with its own Scene (workspace, counters), so that one frame's end of pass can
overlap the next frame's start.  Prints one JSON line per run (wall ms per frame, md5 of
each frame's outputs).  Usage: pipeline_probe.py [K] [ROUNDS]
Env: SLOTS (frames in flight in the "pipe" mode, default 2), LAUNCH=blocks_per_cu,threads
(grt_set_launch_config), MODES (default "seq,pipe")."""
import os
import hashlib
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import gr_raytracer_amd as g  # noqa: E402
from gr_raytracer_amd import _lib as L  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dev = torch.device("cuda:0")
lib = L.lib()
if os.environ.get("LAUNCH"):
    bpc, thr = (int(v) for v in os.environ["LAUNCH"].split(","))
    L.check(lib.grt_set_launch_config(bpc, thr), "grt_set_launch_config")
F = int(os.environ.get("SLOTS", "2"))
MODES = os.environ.get("MODES", "seq,pipe").split(",")
opts = bench.c2_opts(g)
hs = g.HostScene(str(ROOT / "tests/golden/scenes/schwarzschild.toml"), opts, str(ROOT / "tests/golden"))
scenes = [g.Scene(hs.desc_ptr(), keepalive=hs) for _ in range(F)]
n = opts.height * opts.width
outs = [(torch.empty((n, 4), dtype=torch.float32, device=dev), torch.empty(n, dtype=torch.uint8, device=dev),
         torch.empty(n, dtype=torch.uint8, device=dev), torch.zeros(4, dtype=torch.int64, device=dev))
        for _ in range(F)]
streams = [torch.cuda.Stream(dev) for _ in range(F)]


def frame(j, stream):
    x, c, s, st = outs[j]
    L.check(lib.grt_render_pixels_async(scenes[j]._s, 0, stream.cuda_stream, 0, 0, opts.height, opts.width,
                                        x.data_ptr(), c.data_ptr(), s.data_ptr(), None, None, None, st.data_ptr()),
            "grt_render_pixels_async")


def md5(j):
    x, c, _, _ = outs[j]
    return hashlib.md5(x.cpu().numpy().tobytes() + c.cpu().numpy().tobytes()).hexdigest()[:12]


def run(mode):
    for o in outs:
        o[3].zero_()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(K):
        if mode == "seq":
            frame(0, streams[0])
        else:
            frame(k % F, streams[k % F])
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    acc = sum(int(o[3][0]) for o in outs)
    return {"mode": mode, "slots": F if mode == "pipe" else 1, "launch": os.environ.get("LAUNCH", ""), "frames": K,
            "ms_per_frame": dt / K * 1e3, "steps_per_s": acc / dt,
            "md5": [md5(j) for j in range(F if mode == "pipe" else 1)]}


for j in range(F):
    frame(j, streams[j])
    torch.cuda.synchronize(dev)
for _ in range(ROUNDS):
    for mode in MODES:
        print(json.dumps(run(mode)), flush=True)
