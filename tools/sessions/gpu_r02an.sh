#!/bin/bash
# r02an: Schwarzschild RHS divisions without scaling in the fast path (ns) vs head: C2/C3 frames (md5 must
# match), then the GPU parity and whole-frame tests on the ns build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02an
mkdir -p "$OUT"
timeout -k 10 500 python3 -u tools/time_variants.py head ns head ns > "$OUT/c2c3_ab.jsonl" 2> "$OUT/c2c3_ab.err" || { tail -20 "$OUT/c2c3_ab.err" >&2; cat "$OUT/c2c3_ab.jsonl" >&2; exit 1; }
cat "$OUT/c2c3_ab.jsonl" >&2
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_parity.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_parity.log" >&2
exit $rc
