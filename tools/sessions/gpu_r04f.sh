#!/bin/bash
# r04f: PMC passes with the record hand-off (C2 + memory pass, C3, C4 shard 2/8), then the
# whole 4096^2 C4 frame in one launch (bench.py --workload c4; a heartbeat line a minute)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
MEMPASS=1 bash tools/run_pmc.sh r04f_c2 c2 >&2 || exit 1
bash tools/run_pmc.sh r04f_c3 c3 >&2 || exit 1
bash tools/run_pmc.sh r04f_c4 c4 >&2 || exit 1
OUT=gpurun_out/r04f; mkdir -p $OUT
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
timeout -k 10 600 python3 bench.py --workload c4 --steps 1 --warmup 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err
rc=$?
kill $HB
[ $rc -eq 0 ] || { tail -20 $OUT/bench_c4.err >&2; exit 1; }
cut -c1-700 $OUT/bench_c4.json >&2
