#!/bin/bash
# r04m: validation of this build: the whole GPU suite, then C4 shard 2 of 8 (time, md5)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r04m; mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log >&2; exit 1; }
tail -3 $OUT/pytest_gpu.log >&2
timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 >> $OUT/c4_shard2.jsonl 2> $OUT/c4.err || { tail -20 $OUT/c4.err >&2; exit 1; }
cut -c1-400 $OUT/c4_shard2.jsonl >&2
