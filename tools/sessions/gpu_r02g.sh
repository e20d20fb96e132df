#!/bin/bash
# r02g: PMC passes of the current device code: C2 frame (bench's traffic figure) and the
# C4 1/8 shard 2 with the long-ray hand-off (integrate + tail kernels), memory pass included.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
MEMPASS=1 bash tools/run_pmc.sh r02g_c2 c2 || exit 1
echo c2 done >&2
MEMPASS=1 PASS_TIMEOUT=150 bash tools/run_pmc.sh r02g_c4 c4 || exit 1
echo c4 done >&2
