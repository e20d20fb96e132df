#!/bin/bash
# r04j: speculative attempt A/B on C2 and C3: d0 = off, s1 = straight-line sincos only,
# d1 = sincos + range-checked divisions (HEAD default), d1b = d1 with a scheduling barrier
# per RHS; base = the previous commit (C3 md5 reference)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04j; mkdir -p $OUT
timeout -k 10 120 python3 -u -m pytest -x -q --timeout 100 tests/test_gpu_parity.py -k division_in_range > $OUT/div.txt 2>&1 || { tail -30 $OUT/div.txt >&2; exit 1; }
tail -2 $OUT/div.txt >&2
GRT_LIB_ALLOW_MISSING=1 timeout -k 10 840 python3 tools/time_variants.py base d0 s1 d1 d1b d0 s1 d1 d1b >> $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
cat $OUT/ab.jsonl >&2
