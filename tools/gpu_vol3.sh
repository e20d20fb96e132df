#!/bin/bash
# GPU session: volumetric parity + timings + kernel trace + march-kernel lane counters.
# Usage (under gpurun, from the repo root): tools/gpu_vol3.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1
mkdir -p "$OUT"
PYT="python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread"
echo "[gpu_vol3] volumetric parity" >&2
timeout -k 10 600 $PYT -v -rA tests/test_gpu_volumetric.py > "$OUT/pytest_vol.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_vol.log" >&2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc, stopping" >&2; exit $rc; fi
echo "[gpu_vol3] volumetric timings" >&2
timeout -k 10 300 python3 tools/vol_time.py 1500 > "$OUT/vol_time.jsonl" 2>&1 || exit 1
cat "$OUT/vol_time.jsonl" >&2
echo "[gpu_vol3] kernel trace" >&2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/vtrace" -o run --output-format csv -- \
  python3 tools/vol_time.py 1500 schwarzschild-volumetric-stony.toml > "$OUT/vtrace.log" 2>&1 || exit 1
echo "[gpu_vol3] march lane counters" >&2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/mlane" -o run \
  --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
  -- python3 tools/vol_time.py 1500 schwarzschild-volumetric-stony.toml > "$OUT/mlane.log" 2>&1 || exit 1
echo "[gpu_vol3] done" >&2
exit $rc
