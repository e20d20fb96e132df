#!/bin/bash
# r02c: full GPU suite + smoke + bench + bench kernel trace (gpu_round.sh), then the C5 section
# timing and its kernel + memory-copy trace (device-side adaptive pass).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_round.sh r02c || exit $?
OUT=gpurun_out/r02c
timeout -k 10 300 python3 tools/c5_time.py > "$OUT/c5.log" 2>&1 || exit 1
cat "$OUT/c5.log" >&2
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/c5trace" -o run --output-format csv -- \
  python3 tools/c5_time.py > "$OUT/c5trace.log" 2>&1 || exit 1
echo done >&2
