#!/bin/bash
# r02e: long-ray hand-off (tail kernel) -- bit identity + C4 parity tests, the C2 bench
# (no regression from the refactor), C4 shard 2 with the hand-off off / auto / 2x.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02e
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 240 --timeout-method thread \
  -k "tail or c4 or oracle_built" > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log" >&2; exit 1; }
tail -3 "$OUT/pytest_gpu.log" >&2
timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
cat "$OUT/bench.json" >&2
for T in -1 0 32768; do
  GRT_TAIL=$T timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 >> "$OUT/c4_shards.jsonl" 2>> "$OUT/c4.err" || exit 1
  tail -1 "$OUT/c4_shards.jsonl" >&2
done
echo done >&2
