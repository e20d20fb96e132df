#!/bin/bash
# r02k: full GPU round on the current build (parity suite, smoke, bench, kernel trace),
# then the C2 PMC passes whose summary gives bench's traffic figure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_round.sh r02k || exit $?
MEMPASS=1 bash tools/run_pmc.sh r02k_c2 c2 || exit 1
echo pmc done >&2
