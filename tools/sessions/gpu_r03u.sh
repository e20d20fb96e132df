#!/bin/bash
# r03u: all eight 1/8 row-band shards of C4 (band 16) one after another on one GPU with
# this build: the 8-GPU projection (max shard) and its balance
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03u; mkdir -p $OUT
for s in 0 1 2 3 4 5 6 7; do
  timeout -k 10 200 python3 tools/c4_shard_time.py 8 $s >> $OUT/c4_shards.jsonl 2> $OUT/c4.err || { tail -20 $OUT/c4.err >&2; exit 1; }
  tail -1 $OUT/c4_shards.jsonl | cut -c1-160 >&2
done
