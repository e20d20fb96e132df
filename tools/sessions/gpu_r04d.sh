#!/bin/bash
# r04d: the probe key from the distance above the horizon stop radius (two-ended queue):
# the per-ray record of C4 shard 2, then all eight 1/8 shards (the 8-GPU projection)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04d; mkdir -p $OUT
GRT_LIB=$PWD/variants/rt/libgrt.so timeout -k 10 200 python3 tools/c4_ray_times.py $OUT/c4_rt_s2.npz 2 8 >> $OUT/rt.jsonl 2> $OUT/rt.err || { tail $OUT/rt.err >&2; exit 1; }
cat $OUT/rt.jsonl >&2
for s in 0 1 2 3 4 5 6 7; do
  timeout -k 10 200 python3 tools/c4_shard_time.py 8 $s >> $OUT/c4_shards.jsonl 2> $OUT/c4.err || { tail -20 $OUT/c4.err >&2; exit 1; }
  tail -1 $OUT/c4_shards.jsonl | cut -c1-300 >&2
done
