#!/bin/bash
# r02u: instruction scheduler A/B (default max-occupancy vs max-ilp vs max-memory-clause):
# C2 / C3 frames, then C4 shard 2 of 8; frames must match (md5).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02u
mkdir -p "$OUT"
timeout -k 10 500 python3 tools/time_variants.py base ilp mclause base ilp mclause > "$OUT/c2c3_sched.log" 2>&1 || { cat "$OUT/c2c3_sched.log" >&2; exit 1; }
cat "$OUT/c2c3_sched.log" >&2
SHARD=2 bash tools/gpu_variant_ab.sh r02u base ilp base ilp || exit 1
echo done >&2
