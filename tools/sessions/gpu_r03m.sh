#!/bin/bash
# r03m: C4 shard 2/8 tail experiments: baseline (early off), tail kernel at 2 waves per SIMD
# (variant tw2: 32768 quads, hand-off at 32768 live rays; and at 65536), 1 wave with the
# hand-off at 32768 live rays, and the early hand-off with the reduced polling
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03m
mkdir -p "$OUT"
run() {  # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 > "$OUT/one.json" 2> "$OUT/c4.err" || { tail -20 "$OUT/c4.err" >&2; exit 1; }
  sed "s/^/{\"label\": \"$label\", \"run\": /; s/$/}/" "$OUT/one.json" >> "$OUT/c4_shard2.jsonl"
  echo "$label $(cut -c1-200 "$OUT/one.json")" >&2
}
run base
run tw2 GRT_LIB=$PWD/variants/tw2/libgrt.so
run tw2_65536 GRT_LIB=$PWD/variants/tw2/libgrt.so GRT_TAIL=65536
run tw1_32768 GRT_TAIL=32768
run early_400k_16 GRT_EARLY=400000,16
run early_300k_32 GRT_EARLY=300000,32
