#!/bin/bash
# r05m: claims in 64-item chunks until two grids' worth of lanes before the end, then
# exact (hyb), against exact claims throughout (cur) and the round's starting build
# (main): C3 and C2 alternating, then C5
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r05m; mkdir -p $OUT
export GRT_LIB_ALLOW_MISSING=1
CONFIGS=C3,C2 timeout -k 10 500 python3 tools/time_variants.py main cur hyb main cur hyb >> $OUT/c3c2_ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
cat $OUT/c3c2_ab.jsonl >&2
for v in cur hyb cur hyb; do
  GRT_LIB=$PWD/variants/$v/libgrt.so timeout -k 10 120 python3 -u tools/c5_time.py > $OUT/c5_$v.tmp 2>&1 || { cat $OUT/c5_$v.tmp >&2; exit 1; }
  grep run $OUT/c5_$v.tmp | sed "s/^/$v /" | cut -c1-160 | tee -a $OUT/c5_ab.log >&2
done
