#!/bin/bash
# r02aa: launch-shape neutrality tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02aa
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_launch_config.py -m gpu -q -rA -p no:cacheprovider --timeout 300 \
  --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log" >&2; exit 1; }
tail -3 "$OUT/pytest_gpu.log" >&2
