#!/bin/bash
# r04s: one 64-B record per ray except KerrBL (two records, as before): C2 / C3 A/B
# against the previous commit (md5, time), C4 shard 2, then PMC passes of this build
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r04s; mkdir -p $OUT
GRT_LIB_ALLOW_MISSING=1 timeout -k 10 400 python3 tools/time_variants.py old new old new >> $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
cat $OUT/ab.jsonl >&2
timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 >> $OUT/c4_shard2.jsonl 2> $OUT/c4.err || { tail -20 $OUT/c4.err >&2; exit 1; }
cut -c1-300 $OUT/c4_shard2.jsonl >&2
MEMPASS=1 bash tools/run_pmc.sh r04s_c2 c2 >&2 || exit 1
MEMPASS=1 bash tools/run_pmc.sh r04s_c3 c3 >&2 || exit 1
bash tools/run_pmc.sh r04s_c4 c4 >&2 || exit 1
