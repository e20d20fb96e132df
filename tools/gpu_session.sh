#!/bin/bash
# One GPU-box session built from presets (replaces the per-call one-off scripts of rounds
# 1-5; their commands are in git history).  Run from the repo root under gpurun:
#   tools/gpu_session.sh <tag> <preset>[=arg] ...
# Every step runs under its own time limit, and the session stops at the first failure.
# Outputs go to gpurun_out/<tag>/ (PMC passes to gpurun_out/<tag>_<workload>/).
# Presets:
#   suite                  pytest -m gpu (the whole GPU parity suite)
#   suite=EXPR             pytest -m gpu -k EXPR
#   smoke                  __graft_entry__.smoke()
#   bench                  bench.py (C2 headline line)
#   benchprof              rocprofv3 --kernel-trace --stats of bench.py --steps 5, + tools/kernel_period.py
#   bench_seq              bench.py --inflight 1 (one frame after another)
#   bench_gather           bench.py --self-gather (the multi-GPU gather path in a group of one)
#   bench_c4               bench.py --workload c4 (the whole C4 frame) under rocprofv3 --stats
#   pmc=c2|c3|c4|c4full    PMC passes (tools/run_pmc.sh; c4full: FETCH / WRITE only)
#   shards                 the eight C4 1/8 row-band shards (tools/c4_shard_time.py)
#   ab=V1,V2,...           C2 / C3 frames of variants/<V>/libgrt.so in that order (CONFIGS=C2,C3)
#   ab_c5=V1,V2,...        C5 (adaptive) of each variant in that order
#   ab_c4=V1,V2,...        C4 shard 2 of each variant in that order
#   timeline=V:c2|c5       ray-level schedule of a -DGRT_RAY_TIMES=1 variant (tools/ray_timeline.py)
#   paths=V:c2|c3|c4       code-path counts of a -DGRT_PATH_COUNT=1 variant (tools/path_count.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
variants() { tr ',' ' ' <<< "$1"; }
for step in "$@"; do
  name=${step%%=*}; arg=${step#*=}; [ "$arg" = "$step" ] && arg=
  echo "[session] $step" >&2
  case $name in
    suite)
      if [ -n "$arg" ]; then K=(-k "$arg"); else K=(); fi
      timeout -k 10 800 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests "${K[@]}" \
        > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log >&2; exit 1; }
      tail -3 $OUT/pytest_gpu.log >&2 ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
        || { tail -20 $OUT/smoke.log >&2; exit 1; }
      tail -2 $OUT/smoke.log >&2 ;;
    bench)
      timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err >&2; exit 1; }
      cut -c1-400 $OUT/bench.json >&2 ;;
    benchprof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
        python3 bench.py --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err \
        || { tail -20 $OUT/bench_prof.err >&2; exit 1; }
      python3 tools/kernel_period.py $OUT/prof/run_kernel_trace.csv "integrate_kernel<1, false>" 5 \
        > $OUT/kernel_period.json && cut -c1-600 $OUT/kernel_period.json >&2 ;;
    bench_seq)
      timeout -k 10 600 python3 bench.py --inflight 1 > $OUT/bench_seq.json 2> $OUT/bench_seq.err \
        || { tail -20 $OUT/bench_seq.err >&2; exit 1; }
      cut -c1-400 $OUT/bench_seq.json >&2 ;;
    bench_gather)
      MASTER_PORT=29533 timeout -k 10 600 python3 bench.py --self-gather --no-cpu-baseline \
        > $OUT/bench_gather.json 2> $OUT/bench_gather.err || { tail -20 $OUT/bench_gather.err >&2; exit 1; }
      cut -c1-400 $OUT/bench_gather.json >&2 ;;
    bench_c4)
      timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- \
        python3 bench.py --workload c4 --steps 1 --warmup 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err \
        || { tail -20 $OUT/bench_c4.err >&2; exit 1; }
      grep '^{' $OUT/bench_c4.json | cut -c1-400 >&2 ;;
    pmc)
      case $arg in
        c4full) PASSES="fetch write" PASS_TIMEOUT=330 timeout -k 10 700 bash tools/run_pmc.sh ${TAG}_$arg $arg >&2 || exit 1 ;;
        c4) PASS_TIMEOUT=150 timeout -k 10 700 bash tools/run_pmc.sh ${TAG}_$arg $arg >&2 || exit 1 ;;
        *) MEMPASS=1 timeout -k 10 600 bash tools/run_pmc.sh ${TAG}_$arg $arg >&2 || exit 1 ;;
      esac ;;
    shards)
      for s in 0 1 2 3 4 5 6 7; do
        timeout -k 10 200 python3 tools/c4_shard_time.py 8 $s >> $OUT/c4_shards.jsonl 2> $OUT/c4.err \
          || { tail -20 $OUT/c4.err >&2; exit 1; }
      done
      python3 -c "
import json
for l in open('$OUT/c4_shards.jsonl'):
    d = json.loads(l); print(d['shard'], round(d['kernel_ms'] / 1000, 2), d['md5'])" >&2 ;;
    ab)
      GRT_LIB_ALLOW_MISSING=1 CONFIGS=${CONFIGS:-C2,C3} timeout -k 10 600 python3 tools/time_variants.py $(variants "$arg") \
        >> $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
      cat $OUT/ab.jsonl >&2 ;;
    ab_c5)
      for v in $(variants "$arg"); do
        GRT_LIB_ALLOW_MISSING=1 GRT_LIB=$PWD/variants/$v/libgrt.so timeout -k 10 120 python3 -u tools/c5_time.py \
          > $OUT/c5_$v.tmp 2>&1 || { cat $OUT/c5_$v.tmp >&2; exit 1; }
        grep run $OUT/c5_$v.tmp | sed "s/^/$v /" | cut -c1-200 | tee -a $OUT/c5_ab.log >&2
      done ;;
    ab_c4)
      GRT_LIB_ALLOW_MISSING=1 SHARD=${SHARD:-2} timeout -k 10 900 bash tools/gpu_variant_ab.sh $TAG $(variants "$arg") || exit 1 ;;
    timeline|paths)
      v=${arg%%:*}; m=${arg#*:}
      tool=tools/ray_timeline.py; [ $name = paths ] && tool=tools/path_count.py
      if [ $name = paths ]; then A=($m); else A=($m $OUT/${m}_$v.npz); fi
      GRT_LIB_ALLOW_MISSING=1 GRT_LIB=$PWD/variants/$v/libgrt.so timeout -k 10 200 python3 -u $tool "${A[@]}" \
        > $OUT/${name}_${m}_$v.json 2>&1 || { cat $OUT/${name}_${m}_$v.json >&2; exit 1; }
      grep '^{' $OUT/${name}_${m}_$v.json | cut -c1-400 >&2 ;;
    *) echo "unknown preset $step" >&2; exit 2 ;;
  esac
done
echo "[session] done" >&2
