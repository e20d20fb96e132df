#!/bin/bash
# r03e: render_dist's log lines vs grt's on the max-steps 3000 crop (debug)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03e
mkdir -p "$OUT"
FLAGS="--width=48 --height=40 --camera-position=-16.0,0.0,3.5 --theta=-3.142 --max-steps=3000 --config-file tests/golden/scenes/schwarzschild.toml --resource-root tests/golden"
timeout -k 10 120 gr_raytracer_amd/lib/grt $FLAGS render --filename /tmp/o.png 2> "$OUT/grt.err" || exit 1
PYTHONPATH=$PWD timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
  --master-port=29577 -m gr_raytracer_amd.render_dist --backend=gloo --band-rows=8 $FLAGS render --filename /tmp/d.png 2> "$OUT/dist.err" || exit 1
grep -c "did not hit" "$OUT/grt.err" "$OUT/dist.err" >&2
grep -n "INFO" "$OUT/grt.err" "$OUT/dist.err" >&2
