set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
bash tools/run_pmc.sh r01c_pmc || exit 1
python3 tools/pmc_summary.py gpurun_out/r01c_pmc profiles/r01c_pmc.json || exit 1
mkdir -p gpurun_out/r01c_out
timeout -k 10 200 python3 tools/prof_output.py > gpurun_out/r01c_out/events.json 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r01c_out/trace -o run --output-format csv -- python3 tools/prof_output.py > gpurun_out/r01c_out/trace.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE WRITE_SIZE -d gpurun_out/r01c_out/pmc -o run --output-format csv -- python3 tools/prof_output.py > gpurun_out/r01c_out/pmc.log 2>&1 || exit 1
echo ok
