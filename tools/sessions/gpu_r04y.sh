#!/bin/bash
# r04y: final build: PMC passes of C4 shard 2 of 8, then the whole 4096^2 C4 frame in one
# launch (bench.py --workload c4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
bash tools/run_pmc.sh r04y_c4 c4 >&2 || exit 1
OUT=gpurun_out/r04y; mkdir -p $OUT
timeout -k 10 700 python3 bench.py --workload c4 --steps 1 --warmup 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err >&2; exit 1; }
cut -c1-700 $OUT/bench_c4.json >&2
