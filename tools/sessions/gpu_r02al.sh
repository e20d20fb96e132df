#!/bin/bash
# r02al: OCML fallbacks out of line + 3 waves per SIMD for the non-Kerr-Schild integrate kernels (new) vs head:
# C2/C3 frames, then C4 shard 2 of 8 twice each (Kerr-Schild stays at 2 waves); md5 must match.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02al
mkdir -p "$OUT"
timeout -k 10 500 python3 -u tools/time_variants.py head new head new > "$OUT/c2c3_ab.jsonl" 2> "$OUT/c2c3_ab.err" || { tail -20 "$OUT/c2c3_ab.err" >&2; cat "$OUT/c2c3_ab.jsonl" >&2; exit 1; }
cat "$OUT/c2c3_ab.jsonl" >&2
SHARD=2 bash tools/gpu_variant_ab.sh r02al new head new head || exit 1
echo done >&2
