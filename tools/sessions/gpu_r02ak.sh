#!/bin/bash
# r02ak: OCML fallbacks out of line (noinl; and at 3 waves per SIMD, noinlw3) vs head: C2/C3 frames, then
# C4 shard 2 of 8 (head, noinl); md5 must match.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02ak
mkdir -p "$OUT"
timeout -k 10 500 python3 -u tools/time_variants.py head noinl noinlw3 head noinl noinlw3 > "$OUT/c2c3_ab.jsonl" 2> "$OUT/c2c3_ab.err" || { tail -20 "$OUT/c2c3_ab.err" >&2; cat "$OUT/c2c3_ab.jsonl" >&2; exit 1; }
cat "$OUT/c2c3_ab.jsonl" >&2
SHARD=2 bash tools/gpu_variant_ab.sh r02ak head noinl || exit 1
echo done >&2
