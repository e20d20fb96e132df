#!/bin/bash
# r05o: code-path counts of the integrate kernel (diagnostic build pc, -DGRT_PATH_COUNT=1)
# on C2, C3 and C4 shard 2
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r05o; mkdir -p $OUT
export GRT_LIB_ALLOW_MISSING=1 GRT_LIB=$PWD/variants/pc/libgrt.so
for w in c2 c3 c4; do
  timeout -k 10 200 python3 -u tools/path_count.py $w > $OUT/path_$w.json 2>&1 || { cat $OUT/path_$w.json >&2; exit 1; }
  grep '^{' $OUT/path_$w.json >&2
done
