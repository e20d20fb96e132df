#!/bin/bash
# r02m: C5 wall time with the adaptive pass on the device, its kernel + memory-copy trace
# (no copy between the 1-spp pass and the supersample pass).  (A PC-sampling step that
# followed was refused by the pool and has been removed)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02m
mkdir -p "$OUT"
timeout -k 10 120 python3 tools/c5_time.py > "$OUT/c5.log" 2>&1 || { cat "$OUT/c5.log" >&2; exit 1; }
cat "$OUT/c5.log" >&2
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/c5trace" -o run -- \
  python3 tools/c5_time.py > "$OUT/c5trace.log" 2>&1 || { tail -20 "$OUT/c5trace.log" >&2; exit 1; }
echo "c5 trace done" >&2
exit 0
