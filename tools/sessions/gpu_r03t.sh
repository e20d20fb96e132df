#!/bin/bash
# r03t: C5 (adaptive 4x4, fully on the device) and C3 frame times with this build
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03t; mkdir -p $OUT
timeout -k 10 200 python3 tools/c5_time.py > $OUT/c5.jsonl 2> $OUT/c5.err || { tail -20 $OUT/c5.err >&2; exit 1; }
cat $OUT/c5.jsonl >&2
timeout -k 10 200 python3 tools/prof_target.py c3 > $OUT/c3.txt 2> $OUT/c3.err || { tail -20 $OUT/c3.err >&2; exit 1; }
cut -c1-400 $OUT/c3.txt >&2
