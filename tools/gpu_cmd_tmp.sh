set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r01c_out
timeout -k 10 300 python3 tools/c5_time.py > gpurun_out/r01c_out/c5.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/r01c_out/pmc_fetch -o run --output-format csv -- python3 tools/prof_output.py > gpurun_out/r01c_out/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/r01c_out/pmc_write -o run --output-format csv -- python3 tools/prof_output.py > gpurun_out/r01c_out/pmc_write.log 2>&1 || exit 1
echo ok
