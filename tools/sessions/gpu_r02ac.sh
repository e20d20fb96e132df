#!/bin/bash
# r02ac: C2/C3 A/B of RKF running sums (fold) and divisions-before-sincos (divfirst); frames must match (md5).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02ac
mkdir -p "$OUT"
timeout -k 10 700 python3 -u tools/time_variants.py base fold divfirst folddiv base fold divfirst folddiv > "$OUT/c2c3_ab.jsonl" 2> "$OUT/c2c3_ab.err" || { tail -20 "$OUT/c2c3_ab.err" >&2; cat "$OUT/c2c3_ab.jsonl" >&2; exit 1; }
cat "$OUT/c2c3_ab.jsonl" >&2
echo done >&2
