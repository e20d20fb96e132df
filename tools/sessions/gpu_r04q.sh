#!/bin/bash
# r04q: what the integrate kernel's memory-side writes are: write requests by size and
# atomics (TCC_EA0_*), C2 frame and C4 shard 2
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04q; mkdir -p $OUT
for c in c2 c4; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$c -o run --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum -- python3 tools/prof_target.py $c > $OUT/$c.log 2>&1 || { tail -20 $OUT/$c.log >&2; exit 1; }
done
echo done >&2
