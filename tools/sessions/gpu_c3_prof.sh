#!/bin/bash
# C3 (KerrBL 1500^2) kernel trace and PMC passes. Usage: tools/gpu_c3_prof.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3trace -o run -- python3 tools/prof_target.py c3 > $OUT/c3trace.log 2>&1 || exit 1
bash tools/run_pmc.sh $1/c3pmc c3
