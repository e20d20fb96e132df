#!/bin/bash
# r04e: edge tiles of a capped-probe region boosted in the tile order: all eight C4 1/8
# shards, the per-ray record of shard 2, then the whole 4096^2 C4 frame in one launch
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04e; mkdir -p $OUT
for s in 0 1 2 3 4 5 6 7; do
  timeout -k 10 200 python3 tools/c4_shard_time.py 8 $s >> $OUT/c4_shards.jsonl 2> $OUT/c4.err || { tail -20 $OUT/c4.err >&2; exit 1; }
  tail -1 $OUT/c4_shards.jsonl | cut -c1-220 >&2
done
GRT_LIB=$PWD/variants/rt/libgrt.so timeout -k 10 200 python3 tools/c4_ray_times.py $OUT/c4_rt_s2.npz 2 8 >> $OUT/rt.jsonl 2> $OUT/rt.err || { tail $OUT/rt.err >&2; exit 1; }
cat $OUT/rt.jsonl >&2
timeout -k 10 500 python3 bench.py --workload c4 --steps 1 --warmup 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err >&2; exit 1; }
cut -c1-600 $OUT/bench_c4.json >&2
