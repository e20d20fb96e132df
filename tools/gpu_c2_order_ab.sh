#!/bin/bash
# C2 A/B of experimental builds (variants/<V>/libgrt.so), alternating in the order given:
# single-launch frames (tools/time_variants.py, md5 checked) and the pipelined bench loop.
# Usage (gpurun, repo root): tools/gpu_c2_order_ab.sh <tag> V1 V2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; shift; mkdir -p $O
export GRT_LIB_ALLOW_MISSING=1
for v in "$@"; do
  CONFIGS=C2 timeout -k 10 200 python3 tools/time_variants.py $v >> $O/c2_single.jsonl 2> $O/c2_single.err || { tail $O/c2_single.err >&2; exit 1; }
  GRT_LIB=$PWD/variants/$v/libgrt.so timeout -k 10 300 python3 bench.py --no-cli-wall --no-fused-check --no-cpu-baseline \
    > $O/bench_$v.json 2> $O/bench_$v.err || { tail $O/bench_$v.err >&2; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'variant': sys.argv[2], 'ms_per_step': round(d['ms_per_step'], 1), 'single_launch_ms': d['roofline'].get('single_launch_ms')}))" $O/bench_$v.json $v >> $O/c2_bench.jsonl
  tail -1 $O/c2_single.jsonl >&2; tail -1 $O/c2_bench.jsonl >&2
done
