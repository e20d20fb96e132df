#!/bin/bash
# r02o: Kerr-Schild derivative quotients with one shared reciprocal refinement (guarded):
# C4 / tail / trajectory GPU tests on the in-tree build, then C4 shard 2 A/B against the
# plain divisions (variants/ksdiv0 vs ksdiv1, and ksdiv2 = + paired k_x, k_y), alternating; md5s must agree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02o
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 240 --timeout-method thread \
  -k "c4 or tail or kerr or trajectory or health" > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log" >&2; exit 1; }
tail -2 "$OUT/pytest_gpu.log" >&2
SHARD=2 bash tools/gpu_variant_ab.sh r02o ksdiv0 ksdiv1 ksdiv2 ksdiv0 ksdiv1 ksdiv2 || exit 1
echo done >&2
