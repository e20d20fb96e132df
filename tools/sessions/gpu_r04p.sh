#!/bin/bash
# r04p: hand-off bytes per launch (tools/handoff_bytes.py) for C2, C3 and C4 shard 2
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04p; mkdir -p $OUT
for c in c2 c3 c4; do
  timeout -k 10 200 python3 tools/handoff_bytes.py $c >> $OUT/handoff.jsonl 2> $OUT/handoff_$c.err || { tail $OUT/handoff_$c.err >&2; exit 1; }
done
cat $OUT/handoff.jsonl >&2
