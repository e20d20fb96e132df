#!/bin/bash
# r03d: hit-pool descriptor in device memory: C3 / C2 frame determinism, frame-sample
# parity, the hit-pool tests, the 2-slot build's parity subset, C2/C3 A/B vs round 2
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03d
mkdir -p "$OUT"
for c in c3 c2; do
  timeout -k 10 300 python3 tools/diag_frames.py $c > "$OUT/diag_$c.jsonl" 2>&1 || { cat "$OUT/diag_$c.jsonl" >&2; exit 1; }
  echo "== $c" >&2; grep -v amdgpu.ids "$OUT/diag_$c.jsonl" >&2
done
GRT_LIB=$PWD/variants/slots2/libgrt.so timeout -k 10 300 python3 tools/diag_frames.py c3 > "$OUT/diag_c3_slots2.jsonl" 2>&1 || exit 1
echo "== c3 slots2" >&2; grep -v amdgpu.ids "$OUT/diag_c3_slots2.jsonl" >&2
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_frames.py tests/test_hit_pool.py tests/test_adaptive_shards.py -m gpu -q -rA \
  -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_sel.log" 2>&1
rc=$?
tail -4 "$OUT/pytest_sel.log" >&2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
GRT_LIB=$PWD/variants/slots2/libgrt.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_volumetric.py tests/test_hit_pool.py tests/test_tail.py tests/test_gpu_frames.py -m gpu -q -rA \
  -p no:cacheprovider --timeout 300 --timeout-method thread -k "not full_pool" > "$OUT/pytest_slots2.log" 2>&1
rc2=$?
tail -4 "$OUT/pytest_slots2.log" >&2
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
timeout -k 10 400 python3 tools/time_variants.py head cur head cur > "$OUT/c2c3_ab.jsonl" 2> "$OUT/ab.err" || { tail -20 "$OUT/ab.err" >&2; exit 1; }
cat "$OUT/c2c3_ab.jsonl" >&2
exit $((rc + rc2))
