#!/bin/bash
# r04aa: final build: the GPU suite, all eight C4 1/8 shards, the whole C4 frame in one launch
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r04aa; mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log >&2; exit 1; }
tail -3 $OUT/pytest_gpu.log >&2
for s in 0 1 2 3 4 5 6 7; do
  timeout -k 10 200 python3 tools/c4_shard_time.py 8 $s >> $OUT/c4_shards.jsonl 2> $OUT/c4.err || { tail -20 $OUT/c4.err >&2; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/c4_shards.jsonl'):
    d=json.loads(l); print(d['shard'], round(d['kernel_ms']/1000,2), d['md5'])
" >&2
timeout -k 10 600 python3 bench.py --workload c4 --steps 1 --warmup 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err >&2; exit 1; }
grep '^{' $OUT/bench_c4.json | cut -c1-400 >&2
