#!/bin/bash
# r04b: two-ended tile queue (priority wave per SIMD takes the longest tiles, the others
# the shortest; probe key from the radius at the cap) and the 64-B final-state / 16-B meta
# records of the integrate -> shade hand-off: C4 shard 2 with / without the two-ended
# queue, the per-ray record of shard 2 with it, C2 / C3 A/B (round 3, this build, record
# constants written at the ray's start), then the whole GPU suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04b; mkdir -p $OUT
for te in 1 0 1; do
  GRT_TWO_ENDED=$te timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 >> $OUT/c4_shard2.jsonl 2> $OUT/c4.err || { tail -20 $OUT/c4.err >&2; exit 1; }
  tail -1 $OUT/c4_shard2.jsonl | cut -c1-400 >&2
done
GRT_LIB=$PWD/variants/rt/libgrt.so timeout -k 10 200 python3 tools/c4_ray_times.py $OUT/c4_rt_s2.npz 2 8 >> $OUT/rt.jsonl 2> $OUT/rt.err || { tail $OUT/rt.err >&2; exit 1; }
cat $OUT/rt.jsonl >&2
GRT_LIB_ALLOW_MISSING=1 timeout -k 10 300 python3 tools/time_variants.py r03 cur fin1 r03 cur fin1 >> $OUT/c2c3_ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
cat $OUT/c2c3_ab.jsonl >&2
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log >&2; exit 1; }
tail -3 $OUT/pytest_gpu.log >&2
