#!/bin/bash
# r02q: C2 tile-queue order A/B (row-major vs probe-ordered), and the per-pixel step
# distribution of the C2 frame.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02q
mkdir -p "$OUT"
timeout -k 10 200 python3 tools/c2_sched_ab.py 0 1 0 1 0 1 > "$OUT/c2_sched_ab.jsonl" 2> "$OUT/c2_sched_ab.err" || { cat "$OUT/c2_sched_ab.err" >&2; exit 1; }
cat "$OUT/c2_sched_ab.jsonl" >&2
