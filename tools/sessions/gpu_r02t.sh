#!/bin/bash
# r02t: instruction-cache counters of the integrate kernels (C2 frame, C3 frame), one
# --pmc pass each
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02t
mkdir -p "$OUT"
for w in c2 c3; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/icache_$w" -o run \
    --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -- python3 tools/prof_target.py $w > "$OUT/icache_$w.log" 2>&1 || { tail -20 "$OUT/icache_$w.log" >&2; exit 1; }
  echo "$w done" >&2
done
