#!/bin/bash
# r04c: the probe keys and tile order of C4 shard 2 (diagnostic build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04c; mkdir -p $OUT
GRT_LIB=$PWD/variants/rt/libgrt.so timeout -k 10 200 python3 tools/c4_probe_order.py $OUT/probe_s2.npz 2 8 2>&1 | tail -3
