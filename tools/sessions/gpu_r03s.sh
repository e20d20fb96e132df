#!/bin/bash
# r03s: the whole C4 frame in one launch: FETCH_SIZE / WRITE_SIZE passes of this build
# (summary written to profiles/ on the box and to gpurun_out/), then bench.py --workload c4
# on one GPU, whose roofline takes its traffic from that summary
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03s; mkdir -p $OUT
( while true; do sleep 50; date >> $OUT/heartbeat.txt; echo tick >&2; done ) &
HB=$!
trap "kill $HB" EXIT
T="python3 tools/prof_target.py c4full"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/c4full/fetch -o run --pmc FETCH_SIZE -- $T > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/c4full/write -o run --pmc WRITE_SIZE -- $T > $OUT/write.log 2>&1 || exit 1
python3 tools/pmc_summary.py $OUT/c4full profiles/r03s_c4full_pmc.json "grt::integrate_kernel<2, false>" \
  "the whole C4 frame in one launch, tools/prof_target.py c4full (4096^2 kerr.toml, 16.8M rays; FETCH/WRITE passes only)" 16777216 > /dev/null || exit 1
cp profiles/r03s_c4full_pmc.json $OUT/
timeout -k 10 500 python3 bench.py --workload c4 --steps 1 --warmup 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err >&2; exit 1; }
cut -c1-600 $OUT/bench_c4.json >&2
