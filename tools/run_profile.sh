#!/bin/bash
# GPU-box profiling session (run from the repo root under gpurun).
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 120 ./tools/fp64_peak > $OUT/fp64_peak.json 2>&1 || exit 1
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1 || exit 1
echo done
