#!/bin/bash
# r02z: probe shortcuts (escape / still-bound decisions after at most 4096 steps):
# schedule + tail tests, then C4 shard 2 with the old and the new probe, alternating,
# and kerr.toml 1000^2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02z
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_schedule.py tests/test_tail.py -m gpu -q -rA -p no:cacheprovider \
  --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log" >&2; exit 1; }
tail -1 "$OUT/pytest_gpu.log" >&2
SHARD=2 bash tools/gpu_variant_ab.sh r02z oldprobe newprobe oldprobe newprobe || exit 1
timeout -k 10 300 python3 tools/kerr_vol_time.py 1000 kerr.toml > "$OUT/kerr_1000.jsonl" 2> "$OUT/kerr_1000.err" || { tail -20 "$OUT/kerr_1000.err" >&2; exit 1; }
cut -c1-300 "$OUT/kerr_1000.jsonl" >&2
