#!/bin/bash
# r02ai: C2 A/B: quick steps as an inner loop (inner) vs back through the loop top (quick); md5 must match.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02ai
mkdir -p "$OUT"
CONFIGS=C2 timeout -k 10 500 python3 -u tools/time_variants.py quick inner quick inner quick inner > "$OUT/c2_ab.jsonl" 2> "$OUT/c2_ab.err" || { tail -20 "$OUT/c2_ab.err" >&2; cat "$OUT/c2_ab.jsonl" >&2; exit 1; }
cat "$OUT/c2_ab.jsonl" >&2
echo done >&2
