#!/bin/bash
# r02w: long-ray hand-off for volumetric Kerr-Schild scenes: tail / volumetric GPU tests,
# then kerr-volumetric-stony at the reference's example size (1000^2) with the hand-off
# off and on, and kerr.toml at that size for comparison.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02w
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_tail.py tests/test_gpu_volumetric.py -m gpu -q -rA -p no:cacheprovider \
  --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log" >&2; exit 1; }
tail -2 "$OUT/pytest_gpu.log" >&2
GRT_TAIL=0 timeout -k 10 300 python3 tools/kerr_vol_time.py 1000 kerr-volumetric-stony.toml >> "$OUT/kerr_1000.jsonl" 2> "$OUT/kerr_1000.err" || { tail -20 "$OUT/kerr_1000.err" >&2; exit 1; }
tail -1 "$OUT/kerr_1000.jsonl" >&2
timeout -k 10 300 python3 tools/kerr_vol_time.py 1000 kerr-volumetric-stony.toml kerr.toml >> "$OUT/kerr_1000.jsonl" 2> "$OUT/kerr_1000.err" || { tail -20 "$OUT/kerr_1000.err" >&2; exit 1; }
tail -2 "$OUT/kerr_1000.jsonl" >&2
