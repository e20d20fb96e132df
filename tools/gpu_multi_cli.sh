# grt --gpus 1 (the native multi-GPU path, one-rank RCCL) on C2 (1 spp) and C5, and plain grt
# on C2; the two C2 PNGs must be byte-identical.  Usage (gpurun, repo root): tools/gpu_multi_cli.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06s}; mkdir -p $O
T=$(mktemp -d); printf '\n[adaptive_sampling]\nenabled = false\n' | cat tests/golden/scenes/schwarzschild.toml - > $T/c2.toml
A="--width=1500 --height=1500 --camera-position=-16.0,0.0,3.5 --theta=-3.142 --psi=0.0 --phi=0.0 --max-steps=100000 --resource-root tests/golden"
timeout -k 10 120 gr_raytracer_amd/lib/grt --gpus 1 $A --config-file $T/c2.toml render --filename $T/c2.png > $O/grt_gpus1.log 2>&1 || exit 1
timeout -k 10 120 gr_raytracer_amd/lib/grt --gpus 1 $A --config-file tests/golden/scenes/schwarzschild.toml render --filename $T/c5.png > $O/grt_gpus1_c5.log 2>&1 || exit 1
timeout -k 10 120 gr_raytracer_amd/lib/grt $A --config-file $T/c2.toml render --filename $T/c2s.png > $O/grt_single.log 2>&1 || exit 1
cmp $T/c2.png $T/c2s.png && echo "png identical" >> $O/grt_gpus1.log
