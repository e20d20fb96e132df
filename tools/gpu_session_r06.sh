O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 720 python -u -m pytest -v --durations=15 --timeout 400 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as e; e.smoke()" > $O/smoke.log 2>&1 || exit 1
tools/gpu_profile_bench.sh r06h || exit 1
export GRT_LIB_ALLOW_MISSING=1
CONFIGS=C3 timeout -k 10 200 python -u tools/time_variants.py exact nowin exact nowin > gpurun_out/r06h/c3_window_ab.jsonl 2>&1 || exit 1
for i in 1 2; do for v in exact unroll2; do GRT_LIB=$PWD/variants/$v/libgrt.so timeout -k 10 120 python -u tools/vol_time.py 1500 kerr-bl-volumetric-stony.toml | sed "s/^/$v /" >> gpurun_out/r06h/vol_unroll_ab.jsonl || exit 1; done; done
echo done
