#!/bin/bash
# r05g: C4 with the widened Kerr-Schild fast path: all eight 1/8 shards, the whole frame in
# one launch (bench.py --workload c4), PMC passes of integrate_kernel<2, false> on shard 2
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r05g; mkdir -p $OUT
for s in 0 1 2 3 4 5 6 7; do
  timeout -k 10 200 python3 tools/c4_shard_time.py 8 $s >> $OUT/c4_shards.jsonl 2> $OUT/c4.err || { tail -20 $OUT/c4.err >&2; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/c4_shards.jsonl'):
    d=json.loads(l); print(d['shard'], round(d['kernel_ms']/1000,2), d['md5'])
" >&2
PASS_TIMEOUT=150 timeout -k 10 900 bash tools/run_pmc.sh r05g_c4 c4 >&2 || exit 1
timeout -k 10 700 python3 bench.py --workload c4 --steps 1 --warmup 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err >&2; exit 1; }
grep '^{' $OUT/bench_c4.json | cut -c1-600 >&2
