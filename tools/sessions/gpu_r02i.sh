#!/bin/bash
# r02i: exact-count claims for Kerr-Schild; tail / C4 / schedule tests, then C4 shard 2 with
# RKF stages in LDS (variants/base) vs in registers (variants/nokl), alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02i
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 240 --timeout-method thread \
  -k "tail or c4 or oracle_built or schedule" > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log" >&2; exit 1; }
tail -1 "$OUT/pytest_gpu.log" >&2
SHARD=2 bash tools/gpu_variant_ab.sh r02i nokl base nokl base || exit 1
echo done >&2
