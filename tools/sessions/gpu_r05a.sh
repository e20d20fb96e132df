#!/bin/bash
# r05a: range-free arithmetic over the whole exponent plane and the three RHS fast-vs-IEEE
# checks; Kerr-Schild fast-path share of C4 shard 2 before (cap 2^10) and after (host cap
# 2^15); C4 shard 2 A/B round-4 build (head) vs this build (main), alternating (time, md5)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r05a; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_arith.py > $OUT/arith_tests.log 2>&1 || { tail -40 $OUT/arith_tests.log >&2; exit 1; }
tail -3 $OUT/arith_tests.log >&2
timeout -k 10 120 python3 -u tools/arith_map.py $OUT/arith_map.npz 16 > $OUT/arith_map.json 2>&1 || { cat $OUT/arith_map.json >&2; exit 1; }
export GRT_LIB_ALLOW_MISSING=1
for v in cnt10 cnt; do
  GRT_LIB=$PWD/variants/$v/libgrt.so timeout -k 10 200 python3 -u tools/ks_path_count.py 8 2 > $OUT/ks_path_$v.json 2>&1 || { cat $OUT/ks_path_$v.json >&2; exit 1; }
  cat $OUT/ks_path_$v.json >&2
done
SHARD=2 timeout -k 10 500 bash tools/gpu_variant_ab.sh r05a head main head main || exit 1
unset GRT_LIB_ALLOW_MISSING
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tail.py tests/test_gpu_parity.py -k "kerr or c4 or tail or shard" > $OUT/ks_tests.log 2>&1 || { tail -30 $OUT/ks_tests.log >&2; exit 1; }
tail -2 $OUT/ks_tests.log >&2
