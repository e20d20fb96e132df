#!/bin/bash
# r04o: C3 PMC of this build (KerrBL without the range-free divisions) and of the 2-wave
# build (w2: fetch / write only); bench.py default run; rocprofv3 --kernel-trace --stats
# of a short bench run
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r04o; mkdir -p $OUT
MEMPASS=1 bash tools/run_pmc.sh r04o_c3 c3 >&2 || exit 1
for c in FETCH_SIZE WRITE_SIZE SQ_INSTS_VMEM_WR; do
  GRT_LIB=$PWD/variants/w2/libgrt.so GRT_LIB_ALLOW_MISSING=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04o_c3w2/$c -o run --pmc $c -- python3 tools/prof_target.py c3 > gpurun_out/r04o_c3w2_$c.log 2>&1 || { tail gpurun_out/r04o_c3w2_$c.log >&2; exit 1; }
done
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err >&2; exit 1; }
cat $OUT/bench.json >&2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -20 $OUT/bench_prof.err >&2; exit 1; }
echo done >&2
