#!/bin/bash
# r04a: per-ray schedule record of C4 shard 2/8 (diagnostic build variants/rt), then a
# same-box A/B of round 2 (b434f70), round 3 (3ac9c30) and this build (early hand-off
# removed, variants/cur) on C4 shard 2 (x2 alternating) and C2 (x2 alternating)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04a; mkdir -p $OUT
export GRT_LIB_ALLOW_MISSING=1
GRT_LIB=$PWD/variants/rt/libgrt.so timeout -k 10 200 python3 tools/c4_ray_times.py $OUT/c4_rt_s2.npz 2 8 >> $OUT/rt.jsonl 2> $OUT/rt.err
rc=$?; cat $OUT/rt.jsonl >&2
case $rc in 0|1) ;; *) echo "rt run ended with $rc" >&2; tail $OUT/rt.err >&2; exit $rc;; esac
for v in r02 r03 cur r02 r03 cur; do
  GRT_LIB=$PWD/variants/$v/libgrt.so timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 > $OUT/ab.tmp 2> $OUT/ab.err || { tail -20 $OUT/ab.err >&2; exit 1; }
  sed "s/^/{\"variant\": \"$v\", \"r\": /; s/$/}/" $OUT/ab.tmp >> $OUT/c4_ab.jsonl
  tail -1 $OUT/c4_ab.jsonl | cut -c1-200 >&2
done
CONFIGS=C2 timeout -k 10 300 python3 tools/time_variants.py r02 r03 cur r02 r03 cur >> $OUT/c2_ab.jsonl 2> $OUT/c2.err || { tail $OUT/c2.err >&2; exit 1; }
cat $OUT/c2_ab.jsonl >&2
