#!/bin/bash
# r02v: C2 kernel time against rays per lane (last-round fill), twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02v
mkdir -p "$OUT"
for k in 1 2; do
  timeout -k 10 200 python3 tools/c2_rounds.py > "$OUT/c2_rounds_$k.jsonl" 2> "$OUT/c2_rounds.err" || { cat "$OUT/c2_rounds.err" >&2; exit 1; }
  cat "$OUT/c2_rounds_$k.jsonl" >&2
done
