#!/bin/bash
# r02f: hand-off timeline on C4 shard 2 -- 1-wave tail kernel (default), the 2-wave
# variant (variants/tw2, threshold 32768), and the hand-off off; tail tests first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02f
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_tail.py -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  > "$OUT/pytest_tail.log" 2>&1 || { tail -30 "$OUT/pytest_tail.log" >&2; exit 1; }
tail -1 "$OUT/pytest_tail.log" >&2
timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 >> "$OUT/c4.jsonl" 2>> "$OUT/c4.err" || exit 1
tail -1 "$OUT/c4.jsonl" >&2
GRT_LIB=$PWD/variants/tw2/libgrt.so timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 >> "$OUT/c4.jsonl" 2>> "$OUT/c4.err" || exit 1
tail -1 "$OUT/c4.jsonl" >&2
GRT_TAIL=0 timeout -k 10 200 python3 tools/c4_shard_time.py 8 2 >> "$OUT/c4.jsonl" 2>> "$OUT/c4.err" || exit 1
tail -1 "$OUT/c4.jsonl" >&2
echo done >&2
