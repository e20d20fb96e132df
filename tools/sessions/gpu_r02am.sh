#!/bin/bash
# r02am: full GPU round on the final round-2 build (parity suite, smoke, bench, kernel trace),
# the C2 PMC passes whose summary gives bench's traffic figure, then C5 and C3 timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_round.sh r02am || exit $?
MEMPASS=1 bash tools/run_pmc.sh r02am_c2 c2 || exit 1
echo pmc done >&2
OUT=gpurun_out/r02am
timeout -k 10 200 python3 tools/c5_time.py > "$OUT/c5.jsonl" 2> "$OUT/c5.err" || { tail -20 "$OUT/c5.err" >&2; exit 1; }
cat "$OUT/c5.jsonl" >&2
CONFIGS=C3 timeout -k 10 200 python3 tools/time_variants.py > /dev/null 2>&1 || true
echo done >&2
