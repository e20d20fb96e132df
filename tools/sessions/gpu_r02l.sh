#!/bin/bash
# r02l: all eight C4 1/8 row-band shards (the 8-GPU layout) one after another on one GPU,
# then the C4 PMC passes (integrate + tail kernels of shard 2).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02l
mkdir -p "$OUT"
for s in 0 1 2 3 4 5 6 7; do
  timeout -k 10 150 python3 tools/c4_shard_time.py 8 $s >> "$OUT/c4_shards.jsonl" 2> "$OUT/c4_shard_$s.err" || { cat "$OUT/c4_shard_$s.err" >&2; exit 1; }
  tail -1 "$OUT/c4_shards.jsonl" | cut -c1-200 >&2
done
MEMPASS=1 PASS_TIMEOUT=150 bash tools/run_pmc.sh r02l_c4 c4 || exit 1
echo done >&2
