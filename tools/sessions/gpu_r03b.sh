#!/bin/bash
# r03b: C3 frame determinism with the hit-pool build vs the round-2 build
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03b
mkdir -p "$OUT"
timeout -k 10 300 python3 tools/diag_frames.py c3 "$OUT/c3_cur.npz" > "$OUT/diag_cur.jsonl" 2>&1 || { cat "$OUT/diag_cur.jsonl" >&2; exit 1; }
cat "$OUT/diag_cur.jsonl" >&2
GRT_LIB=$PWD/variants/slots2/libgrt.so timeout -k 10 300 python3 tools/diag_frames.py c3 "$OUT/c3_slots2.npz" > "$OUT/diag_slots2.jsonl" 2>&1 || { cat "$OUT/diag_slots2.jsonl" >&2; exit 1; }
cat "$OUT/diag_slots2.jsonl" >&2
GRT_LIB_ALLOW_MISSING=1 GRT_LIB=$PWD/variants/head/libgrt.so timeout -k 10 300 python3 tools/diag_frames.py c3 "$OUT/c3_head.npz" > "$OUT/diag_head.jsonl" 2>&1 || { cat "$OUT/diag_head.jsonl" >&2; exit 1; }
cat "$OUT/diag_head.jsonl" >&2
