#!/bin/bash
# r03k: early hand-off (wave-exit fix, 32-bit lane counters): crop stats, tail tests,
# C4 1/8 shard 2 with the early hand-off off and at three settings
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03k
mkdir -p "$OUT"
timeout -k 10 120 python3 tools/early_debug.py > "$OUT/early_debug.jsonl" 2>&1 || { cat "$OUT/early_debug.jsonl" >&2; exit 1; }
cat "$OUT/early_debug.jsonl" >&2
timeout -k 10 400 python3 -u -m pytest tests/test_tail.py -m gpu -q -rA -p no:cacheprovider --timeout 300 \
  --timeout-method thread --durations=10 > "$OUT/pytest_tail.log" 2>&1
rc=$?
tail -4 "$OUT/pytest_tail.log" >&2
if [ $rc -ne 0 ]; then exit $rc; fi
for e in "0,0" "100000,16" "50000,16" "200000,32"; do
  GRT_EARLY=$e timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 >> "$OUT/c4_shard2.jsonl" 2> "$OUT/c4.err" || { tail -20 "$OUT/c4.err" >&2; exit 1; }
  tail -1 "$OUT/c4_shard2.jsonl" | cut -c1-400 >&2
done
