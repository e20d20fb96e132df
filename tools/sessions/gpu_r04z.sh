#!/bin/bash
# r04z: Kerr-Schild square roots without range steps (sq, GRT_FAST_SQRT_KS) against the
# div_fx-only build (ksfd): the device check, the Kerr-Schild GPU tests, C4 shard 2 A/B
# shard 2 of 8 alternating (time, md5)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r04z; mkdir -p $OUT
timeout -k 10 120 python3 -u -m pytest -x -q --timeout 100 tests/test_gpu_parity.py -k division_in_range > $OUT/div.txt 2>&1 || { tail -30 $OUT/div.txt >&2; exit 1; }
tail -2 $OUT/div.txt >&2
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tail.py tests/test_gpu_parity.py -k "kerr or c4 or tail or shard" > $OUT/ks_tests.log 2>&1 || { tail -30 $OUT/ks_tests.log >&2; exit 1; }
tail -2 $OUT/ks_tests.log >&2
export GRT_LIB_ALLOW_MISSING=1
SHARD=2 timeout -k 10 500 bash tools/gpu_variant_ab.sh r04z ksfd sq ksfd sq || exit 1
