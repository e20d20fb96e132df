# The grt CLI on the C2 command (1 spp): three plain runs (phase line + process wall), then
# one under rocprofv3 --runtime-trace (HIP API, copies, kernels) for the start-up timeline.
# Usage (under gpurun, repo root): tools/gpu_cli_trace.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06m}; mkdir -p $O
T=$(mktemp -d); printf '\n[adaptive_sampling]\nenabled = false\n' | cat tests/golden/scenes/schwarzschild.toml - > $T/c2.toml
ARGS="--width=1500 --height=1500 --camera-position=-16.0,0.0,3.5 --theta=-3.142 --psi=0.0 --phi=0.0 --max-steps=100000 --resource-root tests/golden --config-file $T/c2.toml render --filename $T/c2.png"
for k in 1 2 3; do
  t0=$EPOCHREALTIME
  timeout -k 10 120 gr_raytracer_amd/lib/grt $ARGS > $O/plain$k.log 2>&1 || exit 1
  python3 -c "import sys; print('process wall %.3f s' % (float(sys.argv[2]) - float(sys.argv[1])))" $t0 $EPOCHREALTIME >> $O/plain$k.log
done
timeout -k 10 180 rocprofv3 --runtime-trace --output-format csv -d $O/cli -o run -- gr_raytracer_amd/lib/grt $ARGS > $O/traced.log 2>&1 || exit 1
echo done
