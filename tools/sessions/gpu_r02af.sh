#!/bin/bash
# r02af: C2/C3 A/B of the wave-uniform straight-line sincos (region B) in the Schwarzschild RHS; frames must match (md5).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02af
mkdir -p "$OUT"
timeout -k 10 500 python3 -u tools/time_variants.py headfold sinb headfold sinb headfold sinb > "$OUT/c2c3_ab.jsonl" 2> "$OUT/c2c3_ab.err" || { tail -20 "$OUT/c2c3_ab.err" >&2; cat "$OUT/c2c3_ab.jsonl" >&2; exit 1; }
cat "$OUT/c2c3_ab.jsonl" >&2
echo done >&2
