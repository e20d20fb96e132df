#!/bin/bash
# r03v: C4 shard 2/8 with a longer probe (variants/cap4: 4 x max_radius steps, variants/cap8:
# 8 x, both capped at 131072) against the in-tree build (1.3 x max_radius), alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03v; mkdir -p $OUT
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 > "$OUT/one.json" 2> "$OUT/c4.err" || { tail -20 "$OUT/c4.err" >&2; exit 1; }
  sed "s/^/{\"label\": \"$label\", \"run\": /; s/$/}/" "$OUT/one.json" >> "$OUT/c4_shard2.jsonl"
  echo "$label $(cut -c1-160 "$OUT/one.json")" >&2
}
run base
run cap4 GRT_LIB=$PWD/variants/cap4/libgrt.so
run cap8 GRT_LIB=$PWD/variants/cap8/libgrt.so
run base2
