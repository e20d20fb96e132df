#!/bin/bash
# r05c: KerrBL record momentum out of line (cur) against the build before (main): C3 / C2
# alternating (time, md5); C3 PMC of this build; the C3 GPU parity tests; the ray-level
# schedule of C5's supersample pass (rt: -DGRT_RAY_TIMES=1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r05c; mkdir -p $OUT
CONFIGS=C3,C2 GRT_LIB_ALLOW_MISSING=1 timeout -k 10 400 python3 tools/time_variants.py main cur main cur >> $OUT/c3c2_ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
cat $OUT/c3c2_ab.jsonl >&2
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_frames.py tests/test_gpu_parity.py tests/test_golden_frames.py tests/test_hit_pool.py -k "c3 or kerr_bl or golden or pool" > $OUT/c3_tests.log 2>&1 || { tail -30 $OUT/c3_tests.log >&2; exit 1; }
tail -2 $OUT/c3_tests.log >&2
MEMPASS=1 timeout -k 10 600 bash tools/run_pmc.sh r05c_c3 c3 >&2 || exit 1
GRT_LIB_ALLOW_MISSING=1 GRT_LIB=$PWD/variants/rt/libgrt.so timeout -k 10 200 python3 -u tools/c5_ray_times.py $OUT/c5_ray_times.npz > $OUT/c5_ray_times.json 2>&1 || { cat $OUT/c5_ray_times.json >&2; exit 1; }
cat $OUT/c5_ray_times.json >&2
