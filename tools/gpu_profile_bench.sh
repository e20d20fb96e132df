#!/bin/bash
# The bench line and its rocprofv3 evidence for one build (run under gpurun from the repo
# root): the default bench (BASELINE C2, two frames in flight, fused line, CLI wall-clock,
# CPU baseline), then kernel traces of the bench loop with two frames in flight and with
# one, and the C2 and C5 frames through `grt --gpus 1` (grt_render_frame_multi's one-rank
# RCCL path).
# Usage: tools/gpu_profile_bench.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
for v in "inflight2:--inflight 2" "inflight1:--inflight 1"; do
  name=${v%%:*}; flags=${v#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- \
    python3 -u bench.py --steps 5 --warmup 1 $flags --no-cli-wall --no-fused-check --no-cpu-baseline \
    > $O/bench_$name.json 2> $O/bench_$name.err || exit 1
done
T=$(mktemp -d); printf '\n[adaptive_sampling]\nenabled = false\n' | cat tests/golden/scenes/schwarzschild.toml - > $T/c2.toml
timeout -k 10 120 gr_raytracer_amd/lib/grt --gpus 1 --width=1500 --height=1500 --camera-position=-16.0,0.0,3.5 \
  --theta=-3.142 --psi=0.0 --phi=0.0 --max-steps=100000 --resource-root tests/golden --config-file $T/c2.toml \
  render --filename $T/c2.png > $O/grt_gpus1.log 2>&1 || exit 1
timeout -k 10 120 gr_raytracer_amd/lib/grt --gpus 1 --width=1500 --height=1500 --camera-position=-16.0,0.0,3.5 \
  --theta=-3.142 --psi=0.0 --phi=0.0 --max-steps=100000 --resource-root tests/golden \
  --config-file tests/golden/scenes/schwarzschild.toml render --filename $T/c5.png > $O/grt_gpus1_c5.log 2>&1 || exit 1
echo done
