#!/bin/bash
# r02r: bench.py's C4 strong-scaling mode on one GPU (RCCL group of one) at reduced size,
# CPU baseline included, to exercise the multi-GPU layout's code path on hardware.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02r
mkdir -p "$OUT"
timeout -k 10 400 python3 bench.py --workload c4 --size 1024 --steps 1 --warmup 0 > "$OUT/bench_c4_1024.json" 2> "$OUT/bench_c4.err" || { tail -20 "$OUT/bench_c4.err" >&2; exit 1; }
cat "$OUT/bench_c4_1024.json" >&2
