"""bench.py's C2 line on the GPU (marker `gpu`): two frames in flight, each frame's gather
on its slot's stream through an RCCL group of one (--self-gather), every frame traced in
full.  The C2 frame's accepted-step count is fixed by the integration (bit-exact against
the oracle on crops, md5 fc034258a049 since round 3), so the line's per-frame count must be
exactly it: a frame cut short or counted twice by the slot bookkeeping would change it."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

C2_ACCEPTED_PER_FRAME = 33934152115  # profiles/r05i/c2_ab.jsonl (every round-5 C2 frame)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("inflight,extra", [(2, ["--self-gather"]), (1, [])])
def test_bench_c2_line(gpu, inflight, extra):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    cmd = [sys.executable, str(ROOT / "bench.py"), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
           "--inflight", str(inflight)] + extra
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    cfg = line["config"]
    assert cfg["frames_in_flight"] == inflight
    assert cfg["accepted_steps_per_frame"] == C2_ACCEPTED_PER_FRAME
    assert line["steps"] == 2 and line["n_gpus"] == 1
    r = line["roofline"]
    assert r["kernel_ms"] > 0 and 0 < r["frac"] < 1
    # the per-frame device time and the wall time per frame describe the same run
    assert abs(r["kernel_ms"] - line["ms_per_step"]) < 0.05 * line["ms_per_step"]
    assert line["value"] == pytest.approx(C2_ACCEPTED_PER_FRAME / (line["ms_per_step"] * 1e-3), rel=1e-9)
