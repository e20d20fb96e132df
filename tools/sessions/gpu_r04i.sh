#!/bin/bash
# r04i: which change breaks C3: base (previous commit), new (both), nolds (no LDS
# Cartesian cache), nocold (no cold attribute on the OCML fallbacks)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04i; mkdir -p $OUT
CONFIGS=C3 GRT_LIB_ALLOW_MISSING=1 timeout -k 10 300 python3 tools/time_variants.py base new nolds nocold nolds nocold >> $OUT/c3_ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
cat $OUT/c3_ab.jsonl >&2
