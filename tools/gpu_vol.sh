#!/bin/bash
# GPU session for the VolumetricDisc path: its parity tests first, then the whole GPU
# suite, the C2 bench line, volumetric frame timings and their kernel trace.
# Usage (under gpurun, from the repo root): tools/gpu_vol.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1
mkdir -p "$OUT"
PYT="python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread"
echo "[gpu_vol] volumetric parity" >&2
timeout -k 10 600 $PYT -x -v -rA tests/test_gpu_volumetric.py > "$OUT/pytest_vol.log" 2>&1
rc=$?
tail -5 "$OUT/pytest_vol.log" >&2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc, stopping" >&2; exit $rc; fi
echo "[gpu_vol] full gpu suite" >&2
timeout -k 10 900 $PYT -q -rA -m gpu tests --deselect tests/test_gpu_volumetric.py > "$OUT/pytest_gpu.log" 2>&1
rc2=$?
tail -3 "$OUT/pytest_gpu.log" >&2
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then echo "pytest rc=$rc2, stopping" >&2; exit $rc2; fi
echo "[gpu_vol] bench" >&2
timeout -k 10 400 python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
cat "$OUT/bench.json" >&2
echo "[gpu_vol] volumetric timings" >&2
timeout -k 10 300 python3 tools/vol_time.py 1500 > "$OUT/vol_time.jsonl" 2>&1 || exit 1
cat "$OUT/vol_time.jsonl" >&2
echo "[gpu_vol] kernel trace of one volumetric frame" >&2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/vtrace" -o run --output-format csv -- \
  python3 tools/vol_time.py 1500 schwarzschild-volumetric-stony.toml > "$OUT/vtrace.log" 2>&1 || exit 1
echo "[gpu_vol] done" >&2
exit $((rc | rc2))
