#!/bin/bash
# r04v: same-box A/B of C4 shard 2 of 8: the build the r04e shard numbers came from
# (e = 24547f8) against the final build of the round (final), alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
export GRT_LIB_ALLOW_MISSING=1
SHARD=2 timeout -k 10 600 bash tools/gpu_variant_ab.sh r04v e final e final || exit 1
