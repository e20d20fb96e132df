#!/bin/bash
# r04l: region-B divisions without range steps (f2, GRT_FAST_DIV, range check ahead of the sincos case) against without (f0),
# C2 / C3 time and md5; the device division check first
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04l; mkdir -p $OUT
timeout -k 10 120 python3 -u -m pytest -x -q --timeout 100 tests/test_gpu_parity.py -k division_in_range > $OUT/div.txt 2>&1 || { tail -30 $OUT/div.txt >&2; exit 1; }
tail -2 $OUT/div.txt >&2
GRT_LIB_ALLOW_MISSING=1 timeout -k 10 600 python3 tools/time_variants.py f0 f2 f0 f2 f0 f2 >> $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err >&2; exit 1; }
cat $OUT/ab.jsonl >&2
