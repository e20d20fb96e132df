#!/bin/bash
# r04u: the whole 4096^2 C4 frame in one launch with the final build of the round
# (bench.py --workload c4; a heartbeat line a minute)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r04u; mkdir -p $OUT
timeout -k 10 700 python3 bench.py --workload c4 --steps 1 --warmup 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err >&2; exit 1; }
cut -c1-900 $OUT/bench_c4.json >&2
