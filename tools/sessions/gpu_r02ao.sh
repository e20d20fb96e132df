#!/bin/bash
# r02ao: C2/C3 A/B: max-ilp scheduler (ilp) and no unit-step attempt copy (nounit) vs head; md5 must match.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02ao
mkdir -p "$OUT"
timeout -k 10 500 python3 -u tools/time_variants.py head ilp nounit head ilp nounit > "$OUT/c2c3_ab.jsonl" 2> "$OUT/c2c3_ab.err" || { tail -20 "$OUT/c2c3_ab.err" >&2; cat "$OUT/c2c3_ab.jsonl" >&2; exit 1; }
cat "$OUT/c2c3_ab.jsonl" >&2
echo done >&2
