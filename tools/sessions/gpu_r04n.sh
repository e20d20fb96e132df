#!/bin/bash
# r04n: PMC passes of this build (tools/run_pmc.sh): C2 and C3 frames with the memory
# pass, C4 shard 2 of 8
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
MEMPASS=1 bash tools/run_pmc.sh r04n_c2 c2 >&2 || exit 1
MEMPASS=1 bash tools/run_pmc.sh r04n_c3 c3 >&2 || exit 1
bash tools/run_pmc.sh r04n_c4 c4 >&2 || exit 1
