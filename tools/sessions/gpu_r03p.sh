#!/bin/bash
# r03p: Kerr-Schild drained-queue test every 256 attempts until seen: C4 shard 2/8 traffic
# (FETCH_SIZE / WRITE_SIZE passes), time and md5
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03p_c4; mkdir -p $OUT
T="python3 tools/prof_target.py c4"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/fetch -o run --pmc FETCH_SIZE -- $T > $OUT/fetch.log 2>&1 || exit 1
echo fetch done >&2
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/write -o run --pmc WRITE_SIZE -- $T > $OUT/write.log 2>&1 || exit 1
echo write done >&2
timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 > $OUT/c4_shard2.jsonl 2> $OUT/c4.err || { tail -20 $OUT/c4.err >&2; exit 1; }
cut -c1-300 $OUT/c4_shard2.jsonl >&2
