#!/bin/bash
# r02ad: ray migration (Kerr-Schild, after the queue drains): bit-identity tests, then
# C4 shard 2 of 8 without / with migration (md5 must match).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02ad
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_tail.py -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > "$OUT/pytest_tail.log" 2>&1 || { tail -30 "$OUT/pytest_tail.log" >&2; exit 1; }
tail -3 "$OUT/pytest_tail.log" >&2
for m in 16 0 32; do
  GRT_MIGRATE=$m timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 >> "$OUT/c4_migrate.jsonl" 2> "$OUT/c4_$m.err" || { tail -20 "$OUT/c4_$m.err" >&2; exit 1; }
  tail -1 "$OUT/c4_migrate.jsonl" >&2
done
echo done >&2
