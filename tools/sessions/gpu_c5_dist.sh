#!/bin/bash
# C5 (stock schwarzschild.toml: adaptive 4x4) through the single-GPU grt binary and the
# multi-GPU render_dist command (world of one here): wall-clock and byte equality.
# Usage (repo root, under gpurun): tools/gpu_c5_dist.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1
mkdir -p "$OUT"
FLAGS="--width=1500 --height=1500 --camera-position=-16.0,0.0,3.5 --theta=-3.142 --psi=0.0 --phi=0.0 --max-steps=100000 --config-file tests/golden/scenes/schwarzschild.toml --resource-root tests/golden"
timeout -k 10 200 gr_raytracer_amd/lib/grt $FLAGS render --filename "$OUT/c5_grt.png" > "$OUT/c5_grt.log" 2>&1 || exit 1
timeout -k 10 300 python3 -m gr_raytracer_amd.render_dist $FLAGS render --filename "$OUT/c5_dist.png" > "$OUT/c5_dist.log" 2>&1 || exit 1
cat "$OUT/c5_grt.log" "$OUT/c5_dist.log" >&2
cmp "$OUT/c5_grt.png" "$OUT/c5_dist.png" && echo "[c5] PNG byte-identical" | tee -a "$OUT/c5_dist.log" >&2
