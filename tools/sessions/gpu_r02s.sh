#!/bin/bash
# r02s: which counters the gfx950 SQ/SQC blocks offer (instruction fetch / cache)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02s
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || { tail -20 "$OUT/counters.txt" >&2; exit 1; }
grep -i -E "ICACHE|IFETCH|SQC_|INST_LEVEL|WAIT_INST" "$OUT/counters.txt" | head -80 >&2
