#!/bin/bash
# A/B of integrate-kernel variants on a C4 1/8 shard (SHARD=, default 0).
# Usage (repo root, under gpurun): tools/gpu_variant_ab.sh <tag> variant...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for v in "$@"; do
  echo "[ab] $v" >&2
  GRT_LIB=$PWD/variants/$v/libgrt.so timeout -k 10 200 python3 tools/c4_shard_time.py 8 ${SHARD:-0} > "$OUT/ab_$v.tmp" 2>&1 || { cat "$OUT/ab_$v.tmp" >&2; exit 1; }
  sed "s/^/$v /" "$OUT/ab_$v.tmp" | tee -a "$OUT/variant_ab.log" >&2
done
