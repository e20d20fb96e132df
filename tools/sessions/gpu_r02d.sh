#!/bin/bash
# r02d: the CLI failed-pixel log test (sub-sample failures included), C5 section timing +
# kernel/memory-copy trace, and the C4 tail measurement (shard 2 steps, lone longest ray).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02d
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 240 --timeout-method thread \
  -k "failed_pixels or failed_subsamples" > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log" >&2; exit 1; }
tail -3 "$OUT/pytest_gpu.log" >&2
timeout -k 10 300 python3 tools/c5_time.py > "$OUT/c5.log" 2>&1 || exit 1
cat "$OUT/c5.log" >&2
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/c5trace" -o run --output-format csv -- \
  python3 tools/c5_time.py > "$OUT/c5trace.log" 2>&1 || exit 1
timeout -k 10 400 python3 tools/c4_tail_probe.py r02d 2 > "$OUT/c4_tail.log" 2>&1 || { cat "$OUT/c4_tail.log" >&2; exit 1; }
cat "$OUT/c4_tail.log" >&2
echo done >&2
