#!/bin/bash
# r03n: PMC passes of the current build: C2 frame (+ memory pass), C3 frame, C4 shard 2/8
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
MEMPASS=1 bash tools/run_pmc.sh r03n_c2 c2 >&2 || exit 1
bash tools/run_pmc.sh r03n_c3 c3 >&2 || exit 1
bash tools/run_pmc.sh r03n_c4 c4 >&2 || exit 1
