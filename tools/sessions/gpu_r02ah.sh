#!/bin/bash
# r02ah: C2 A/B of the Schwarzschild quick far-field step (quick) vs without (noquick); md5 must match.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02ah
mkdir -p "$OUT"
CONFIGS=C2 timeout -k 10 500 python3 -u tools/time_variants.py noquick quick noquick quick noquick quick > "$OUT/c2_ab.jsonl" 2> "$OUT/c2_ab.err" || { tail -20 "$OUT/c2_ab.err" >&2; cat "$OUT/c2_ab.jsonl" >&2; exit 1; }
cat "$OUT/c2_ab.jsonl" >&2
echo done >&2
