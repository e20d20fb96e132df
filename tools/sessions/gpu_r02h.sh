#!/bin/bash
# r02h: RKF stages in LDS for the Kerr-Schild integrate kernel -- tail + C4 parity tests,
# C4 shard 2 timing; C2/C3 A/B of the LDS stages for Schwarzschild/KerrBL (variants/klall).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02h
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 240 --timeout-method thread \
  -k "tail or c4 or oracle_built or schedule" > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log" >&2; exit 1; }
tail -1 "$OUT/pytest_gpu.log" >&2
timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 >> "$OUT/c4.jsonl" 2>> "$OUT/c4.err" || exit 1
tail -1 "$OUT/c4.jsonl" >&2
timeout -k 10 500 python3 tools/time_variants.py base klall base klall > "$OUT/variants.log" 2>&1 || { cat "$OUT/variants.log" >&2; exit 1; }
cat "$OUT/variants.log" >&2
echo done >&2
