#!/bin/bash
# r03r (as r03o, after the drained-queue poll change): HBM traffic of the whole C4 frame in one launch (bench.py --workload c4 on one GPU):
# the FETCH_SIZE and WRITE_SIZE passes only (the other counters come from the shard, r03n_c4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03r_c4full; mkdir -p $OUT
T="python3 tools/prof_target.py c4full"
# heartbeat: a pass runs ~5 minutes without output
( while true; do sleep 50; date >> $OUT/heartbeat.txt; echo tick >&2; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $OUT/fetch -o run --pmc FETCH_SIZE -- $T > $OUT/fetch.log 2>&1 || exit 1
echo fetch done >&2
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $OUT/write -o run --pmc WRITE_SIZE -- $T > $OUT/write.log 2>&1 || exit 1
echo write done >&2
