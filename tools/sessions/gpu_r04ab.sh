#!/bin/bash
# r04ab: final build: smoke(), the C5 adaptive frame (tools/c5_time.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04ab; mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log >&2; exit 1; }
tail -1 $OUT/smoke.log >&2
timeout -k 10 300 python3 tools/c5_time.py > $OUT/c5.jsonl 2> $OUT/c5.err || { tail -20 $OUT/c5.err >&2; exit 1; }
cut -c1-400 $OUT/c5.jsonl >&2
