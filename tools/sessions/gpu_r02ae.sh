#!/bin/bash
# r02ae: full GPU round on the running-sum + straight-line sincos build (parity suite, smoke, bench, kernel trace),
# then the C2 PMC passes whose summary gives bench's traffic figure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_round.sh r02ae || exit $?
MEMPASS=1 bash tools/run_pmc.sh r02ae_c2 c2 || exit 1
echo pmc done >&2
