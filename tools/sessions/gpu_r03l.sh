#!/bin/bash
# r03l: C2/C3 A/B of the committed build (base) against the working tree (cur: OCML sincos
# fallback returned by value, scalar ray counter), and the per-ray steps of C4 shard 2/8
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03l
mkdir -p "$OUT"
timeout -k 10 400 python3 tools/time_variants.py base cur base cur > "$OUT/c2c3_ab.jsonl" 2> "$OUT/ab.err" || { tail -20 "$OUT/ab.err" >&2; exit 1; }
cat "$OUT/c2c3_ab.jsonl" >&2
timeout -k 10 200 python3 tools/step_hist.py c4 8 2 > "$OUT/step_hist.json" 2> "$OUT/hist.err" || { tail -20 "$OUT/hist.err" >&2; exit 1; }
cat "$OUT/step_hist.json" >&2
mv gpurun_out/steps_c4_8_2.npy gpurun_out/stop_c4_8_2.npy "$OUT/"
