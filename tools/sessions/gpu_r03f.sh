#!/bin/bash
# r03f: grt vs render_dist log lines on the max-steps 3000 crop (kept for host-side diff
# against the oracle), then the full GPU round (suite, smoke, bench, kernel trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03f
mkdir -p "$OUT"
FLAGS="--width=48 --height=40 --camera-position=-16.0,0.0,3.5 --theta=-3.142 --max-steps=3000 --config-file tests/golden/scenes/schwarzschild.toml --resource-root tests/golden"
timeout -k 10 120 gr_raytracer_amd/lib/grt $FLAGS render --filename /tmp/o.png 2> "$OUT/grt.err" || exit 1
PYTHONPATH=$PWD timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
  --master-port=29577 -m gr_raytracer_amd.render_dist --backend=gloo --band-rows=8 $FLAGS render --filename /tmp/d.png 2> "$OUT/dist.err" || exit 1
PYTHONPATH=$PWD timeout -k 10 200 python3 -m gr_raytracer_amd.render_dist $FLAGS render --filename /tmp/d1.png 2> "$OUT/dist1.err" || exit 1
grep -c "did not hit" "$OUT/grt.err" "$OUT/dist.err" "$OUT/dist1.err" >&2
bash tools/gpu_round.sh r03f
