mkdir -p gpurun_out/r01e
timeout -k 10 900 python3 -m pytest tests -m gpu -q -rA -p no:cacheprovider > gpurun_out/r01e/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/r01e/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python3 tools/gpu_check.py > gpurun_out/r01e/gpu_check.log 2>&1 || exit 3
cat gpurun_out/r01e/gpu_check.log
exit $rc
