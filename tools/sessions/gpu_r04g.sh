#!/bin/bash
# r04g: C2 / C3 A/B: this commit (base), Cartesian cache in LDS for the 3-wave kernels
# (clds), 2 waves per SIMD for the light kernels (w2)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04g; mkdir -p $OUT
GRT_LIB_ALLOW_MISSING=1 timeout -k 10 500 python3 tools/time_variants.py base clds w2 base clds w2 >> $OUT/c2c3_ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
cat $OUT/c2c3_ab.jsonl >&2
