#!/bin/bash
# r04f: PMC passes with the record hand-off (C2 + memory pass, C3, C4 shard 2/8), then the
# whole 4096^2 C4 frame in one launch (bench.py --workload c4; a heartbeat line a minute)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
MEMPASS=1 bash tools/run_pmc.sh r04f_c2 c2 >&2 || exit 1
MEMPASS=1 bash tools/run_pmc.sh r04f_c3 c3 >&2 || exit 1
bash tools/run_pmc.sh r04f_c4 c4 >&2 || exit 1
OUT=gpurun_out/r04f; mkdir -p $OUT
timeout -k 10 600 python3 bench.py --workload c4 --steps 1 --warmup 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err
rc=$?
[ $rc -eq 0 ] || { tail -20 $OUT/bench_c4.err >&2; exit 1; }
cut -c1-700 $OUT/bench_c4.json >&2
GRT_LIB_ALLOW_MISSING=1 timeout -k 10 300 python3 tools/time_variants.py base cnt base cnt >> $OUT/c2c3_cnt_ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
cat $OUT/c2c3_cnt_ab.jsonl >&2
