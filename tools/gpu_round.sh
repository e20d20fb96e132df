#!/bin/bash
# One GPU-box session: GPU parity suite, smoke, bench line, kernel-trace profile of the bench.
# Usage (from the repo root, under gpurun): tools/gpu_round.sh <tag> [pytest -k expr]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1
mkdir -p "$OUT"
KEXPR=${2:-}
echo "[gpu_round] pytest -m gpu" >&2
if [ -n "$KEXPR" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 300 --timeout-method thread --durations=25 -k "$KEXPR" > "$OUT/pytest_gpu.log" 2>&1
else
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 300 --timeout-method thread --durations=25 > "$OUT/pytest_gpu.log" 2>&1
fi
rc=$?
tail -5 "$OUT/pytest_gpu.log" >&2
# a failing assertion (1) still allows the next steps; a crash/timeout does not
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc, stopping" >&2; exit $rc; fi
echo "[gpu_round] smoke" >&2
timeout -k 10 300 python3 -c "import __graft_entry__ as e; e.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
echo "[gpu_round] bench" >&2
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
cat "$OUT/bench.json" >&2
echo "[gpu_round] rocprofv3 kernel trace" >&2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline > "$OUT/trace.log" 2>&1 || exit 1
echo "[gpu_round] done" >&2
exit $rc
