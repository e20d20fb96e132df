#!/bin/bash
# HBM request accounting of one frame (run under gpurun from the repo root): for each
# workload of tools/prof_target.py, one rocprofv3 --pmc pass of the L2 -> memory write
# requests (all, 64-B, atomics) and one of the read requests, each a run of its own
# (counters only with --kernel-trace), then the integrate -> shade hand-off of the same
# frame (tools/handoff_bytes.py).  Summaries: tools/requests_summary.py.
# Usage: tools/gpu_requests.sh <tag> c2 [c3 ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for w in "$@"; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $O/${w}_wr -o run \
    --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum -- python3 tools/prof_target.py $w \
    > $O/${w}_wr.log 2>&1 || { tail -20 $O/${w}_wr.log >&2; exit 1; }
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $O/${w}_rd -o run \
    --pmc TCC_EA0_RDREQ_sum -- python3 tools/prof_target.py $w \
    > $O/${w}_rd.log 2>&1 || { tail -20 $O/${w}_rd.log >&2; exit 1; }
  timeout -k 10 240 python3 tools/handoff_bytes.py $w > $O/${w}_handoff.json 2> $O/${w}_handoff.err \
    || { tail -20 $O/${w}_handoff.err >&2; exit 1; }
  echo "[requests] $w done" >&2
done
