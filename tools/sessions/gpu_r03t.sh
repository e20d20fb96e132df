#!/bin/bash
# r03t: C5 (adaptive 4x4, fully on the device) and C3 frame times with this build; C4 shard 2
# with the early kernel on 16 CUs but no ray ever handed early (the cost of the split)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03t; mkdir -p $OUT
timeout -k 10 200 python3 tools/c5_time.py > $OUT/c5.jsonl 2> $OUT/c5.err || { tail -20 $OUT/c5.err >&2; exit 1; }
cat $OUT/c5.jsonl >&2
timeout -k 10 200 python3 tools/prof_target.py c3 > $OUT/c3.txt 2> $OUT/c3.err || { tail -20 $OUT/c3.err >&2; exit 1; }
cut -c1-400 $OUT/c3.txt >&2
# the cost of the CU split alone: early kernel on 16 CUs, threshold never reached
GRT_EARLY=1000000000,16 timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 > $OUT/c4_split_only.jsonl 2> $OUT/c4.err || { tail -20 $OUT/c4.err >&2; exit 1; }
cut -c1-300 $OUT/c4_split_only.jsonl >&2
