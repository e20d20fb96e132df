#!/bin/bash
# r02x: kerr.toml at 1000^2: hand-off timeline and the frame's long-ray count
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02x
mkdir -p "$OUT"
timeout -k 10 300 python3 tools/kerr_vol_time.py 1000 kerr.toml > "$OUT/kerr_1000.jsonl" 2> "$OUT/kerr_1000.err" || { tail -20 "$OUT/kerr_1000.err" >&2; exit 1; }
cat "$OUT/kerr_1000.jsonl" >&2
