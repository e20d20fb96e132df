#!/bin/bash
# r04r: one 64-B record per ray (meta folded in, observer energy recomputed by the shade
# kernel, steps written straight to the output): C2 / C3 A/B against the previous commit
# (md5, time), the GPU suite, C4 shard 2 (md5, time)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r04r; mkdir -p $OUT
GRT_LIB_ALLOW_MISSING=1 timeout -k 10 400 python3 tools/time_variants.py old new old new >> $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
cat $OUT/ab.jsonl >&2
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log >&2; exit 1; }
tail -3 $OUT/pytest_gpu.log >&2
timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 >> $OUT/c4_shard2.jsonl 2> $OUT/c4.err || { tail -20 $OUT/c4.err >&2; exit 1; }
cut -c1-300 $OUT/c4_shard2.jsonl >&2
