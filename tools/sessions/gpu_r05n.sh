#!/bin/bash
# r05n: final build: GPU suite, smoke(), bench.py (C2, traffic from profiles/r05j_c2_pmc.json) and bench.py
# --workload c4 (the whole frame, traffic from profiles/r05k_c4full_pmc.json), the latter
# also under rocprofv3 --kernel-trace --stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r05n; mkdir -p $OUT
timeout -k 10 800 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log >&2; exit 1; }
tail -3 $OUT/pytest_gpu.log >&2
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log >&2; exit 1; }
tail -2 $OUT/smoke.log >&2
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err >&2; exit 1; }
cut -c1-300 $OUT/bench.json >&2
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --steps 1 --warmup 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err >&2; exit 1; }
grep '^{' $OUT/bench_c4.json | cut -c1-300 >&2
