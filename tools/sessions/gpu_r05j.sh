#!/bin/bash
# r05j: final build of round 5: GPU suite, smoke(), bench.py default, rocprofv3
# --kernel-trace --stats of a short bench run, PMC of the C2 and C3 integrate kernels and of
# C4 shard 2
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r05j; mkdir -p $OUT
timeout -k 10 800 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log >&2; exit 1; }
tail -3 $OUT/pytest_gpu.log >&2
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log >&2; exit 1; }
tail -3 $OUT/smoke.log >&2
MEMPASS=1 timeout -k 10 600 bash tools/run_pmc.sh r05j_c2 c2 >&2 || exit 1
timeout -k 10 400 bash tools/run_pmc.sh r05j_c3 c3 >&2 || exit 1
PASS_TIMEOUT=150 timeout -k 10 700 bash tools/run_pmc.sh r05j_c4 c4 >&2 || exit 1
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err >&2; exit 1; }
cut -c1-600 $OUT/bench.json >&2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -20 $OUT/bench_prof.err >&2; exit 1; }
echo done >&2
