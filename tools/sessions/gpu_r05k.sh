#!/bin/bash
# r05k: final build of round 5: C3 against the round's starting build (main) alternating
# and the C3 PMC (KerrBL claims chunks until the end of its queue); C4: all eight 1/8
# shards, HBM traffic of the whole frame in one launch (FETCH / WRITE passes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r05k; mkdir -p $OUT
CONFIGS=C3 GRT_LIB_ALLOW_MISSING=1 timeout -k 10 300 python3 tools/time_variants.py main fin main fin >> $OUT/c3_ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
cat $OUT/c3_ab.jsonl >&2
timeout -k 10 400 bash tools/run_pmc.sh r05k_c3 c3 >&2 || exit 1
for s in 0 1 2 3 4 5 6 7; do
  timeout -k 10 200 python3 tools/c4_shard_time.py 8 $s >> $OUT/c4_shards.jsonl 2> $OUT/c4.err || { tail -20 $OUT/c4.err >&2; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/c4_shards.jsonl'):
    d=json.loads(l); print(d['shard'], round(d['kernel_ms']/1000,2), d['md5'])
" >&2
PASSES="fetch write" PASS_TIMEOUT=330 timeout -k 10 700 bash tools/run_pmc.sh r05k_c4full c4full >&2 || exit 1
echo done >&2
