#!/bin/bash
# r02aj: C2 A/B: head (b134680) vs cur (+ no unit-step re-ballot after a quick step) vs sinac (+ straight-line sincos for regions A and C); md5 must match.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02aj
mkdir -p "$OUT"
CONFIGS=C2 timeout -k 10 500 python3 -u tools/time_variants.py head cur sinac head cur sinac head cur sinac > "$OUT/c2_ab.jsonl" 2> "$OUT/c2_ab.err" || { tail -20 "$OUT/c2_ab.err" >&2; cat "$OUT/c2_ab.jsonl" >&2; exit 1; }
cat "$OUT/c2_ab.jsonl" >&2
echo done >&2
