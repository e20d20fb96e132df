#!/bin/bash
# r02b: device-side adaptive pass -- GPU tests of the adaptive / section / shard paths,
# C5 timing, and a kernel + memory-copy trace of the C5 section (no host copies between
# the 1-spp pass and the supersample pass).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02b
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 300 --timeout-method thread \
  --durations=15 -k "frames or adaptive or section or cli or shard or output or render_dist" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -5 "$OUT/pytest_gpu.log" >&2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc, stopping" >&2; exit $rc; fi
timeout -k 10 300 python3 tools/c5_time.py > "$OUT/c5.log" 2>&1 || exit 1
cat "$OUT/c5.log" >&2
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/c5trace" -o run --output-format csv -- \
  python3 tools/c5_time.py > "$OUT/c5trace.log" 2>&1 || exit 1
echo done >&2
exit $rc
