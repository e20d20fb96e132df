#!/bin/bash
# r03a: GPU suite on the hit-pool build (no 16-candidate cap), the parity tests again on a
# 2-slot build (nearly every candidate through the pool), and C2/C3 kernel time against
# the round-2 build (alternating, frames must be md5-identical).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03a
mkdir -p "$OUT"
echo "[r03a] pytest -m gpu" >&2
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 300 --timeout-method thread \
  --durations=30 > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -5 "$OUT/pytest_gpu.log" >&2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc, stopping" >&2; exit $rc; fi
echo "[r03a] 2-slot build" >&2
GRT_LIB=$PWD/variants/slots2/libgrt.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_volumetric.py tests/test_hit_pool.py tests/test_tail.py tests/test_gpu_fuzz.py -m gpu -q -rA \
  -p no:cacheprovider --timeout 300 --timeout-method thread -k "not full_pool" > "$OUT/pytest_slots2.log" 2>&1
rc2=$?
tail -5 "$OUT/pytest_slots2.log" >&2
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then echo "pytest rc=$rc2, stopping" >&2; exit $rc2; fi
echo "[r03a] C2/C3 A/B" >&2
timeout -k 10 400 python3 tools/time_variants.py head cur head cur > "$OUT/c2c3_ab.jsonl" 2> "$OUT/ab.err" || { tail -20 "$OUT/ab.err" >&2; exit 1; }
cat "$OUT/c2c3_ab.jsonl" >&2
exit $rc
