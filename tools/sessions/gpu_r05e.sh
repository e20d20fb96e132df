#!/bin/bash
# r05e: exact claims for offset lists (ex1, C5's supersample pass) against the build before
# (main): C5 alternating; every list claiming exactly (ex2) on C2; the C5 sub-ray pass's
# ray-level schedule with exact claims (rt)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r05e; mkdir -p $OUT
export GRT_LIB_ALLOW_MISSING=1
for v in main ex1 main ex1; do
  GRT_LIB=$PWD/variants/$v/libgrt.so timeout -k 10 120 python3 -u tools/c5_time.py > $OUT/c5_$v.tmp 2>&1 || { cat $OUT/c5_$v.tmp >&2; exit 1; }
  grep run $OUT/c5_$v.tmp | sed "s/^/$v /" | tee -a $OUT/c5_ab.log >&2
done
CONFIGS=C2 timeout -k 10 400 python3 tools/time_variants.py main ex2 main ex2 >> $OUT/c2_ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
cat $OUT/c2_ab.jsonl >&2
GRT_LIB=$PWD/variants/rt/libgrt.so timeout -k 10 200 python3 -u tools/c5_ray_times.py $OUT/c5_ray_times.npz > $OUT/c5_ray_times.json 2>&1 || { cat $OUT/c5_ray_times.json >&2; exit 1; }
cut -c1-400 $OUT/c5_ray_times.json >&2
