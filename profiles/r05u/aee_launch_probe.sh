mkdir -p gpurun_out/r05u
export GRT_LIB_ALLOW_MISSING=1 GRT_LIB=$PWD/variants/aee/libgrt.so
for b in 1 2 3 6; do
  GRT_BLOCKS_PER_CU=$b timeout -k 10 120 python3 -u tools/c3_det.py gpurun_out/r05u/aee_b$b 3 1 > gpurun_out/r05u/aee_b$b.jsonl 2>&1 || { cat gpurun_out/r05u/aee_b$b.jsonl; exit 1; }
  sed "s/^/b$b /" gpurun_out/r05u/aee_b$b.jsonl | grep run
done
