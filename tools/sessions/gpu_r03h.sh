#!/bin/bash
# r03h: early hand-off stats debugging on the C4 crop
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r03h
timeout -k 10 120 python3 tools/early_debug.py > gpurun_out/r03h/early_debug.jsonl 2>&1; rc=$?
cat gpurun_out/r03h/early_debug.jsonl >&2
exit $rc
