#!/bin/bash
# r05h: drain hand-off to a packed resume launch for Schwarzschild (dr) against this build
# (cur): C2 and C5 alternating (time, md5); ray-level timelines of C2 and of C5's
# supersample pass with (rtdr) and without (rt) the drain hand-off
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r05h; mkdir -p $OUT
export GRT_LIB_ALLOW_MISSING=1
CONFIGS=C2 timeout -k 10 400 python3 tools/time_variants.py cur dr cur dr >> $OUT/c2_ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
cat $OUT/c2_ab.jsonl >&2
for v in cur dr cur dr; do
  GRT_LIB=$PWD/variants/$v/libgrt.so timeout -k 10 120 python3 -u tools/c5_time.py > $OUT/c5_$v.tmp 2>&1 || { cat $OUT/c5_$v.tmp >&2; exit 1; }
  grep run $OUT/c5_$v.tmp | sed "s/^/$v /" | cut -c1-160 | tee -a $OUT/c5_ab.log >&2
done
for v in rt rtdr; do
  for m in c2 c5; do
    GRT_LIB=$PWD/variants/$v/libgrt.so timeout -k 10 200 python3 -u tools/ray_timeline.py $m $OUT/${m}_$v.npz > $OUT/${m}_$v.json 2>&1 || { cat $OUT/${m}_$v.json >&2; exit 1; }
    cut -c1-300 $OUT/${m}_$v.json >&2
  done
done
