#!/bin/bash
# r02p: C2 / C3 frame times of RKF stages parked in LDS for Schwarzschild (kl4s: k1..k4,
# kl2s: k1..k2; both attempt copies) against the default build, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02p
mkdir -p "$OUT"
timeout -k 10 500 python3 tools/time_variants.py base kl4s kl2s base kl4s kl2s > "$OUT/c2_klds_ab.log" 2>&1 || { cat "$OUT/c2_klds_ab.log" >&2; exit 1; }
cat "$OUT/c2_klds_ab.log" >&2
