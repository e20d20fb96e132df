set -o pipefail
mkdir -p gpurun_out/r01i
timeout -k 10 900 python3 tools/time_variants.py base div lds_div > gpurun_out/r01i/variants.log 2>&1; rc=$?
cat gpurun_out/r01i/variants.log
exit $rc
