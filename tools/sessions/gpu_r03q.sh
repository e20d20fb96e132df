#!/bin/bash
# r03q: (1) Kerr-Schild drained-queue test every 256 attempts until seen: C4 shard 2/8
# traffic (FETCH_SIZE / WRITE_SIZE passes), time and md5; (2) the full GPU round of this
# build (suite, smoke, bench, kernel trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/sessions/gpu_r03p.sh || exit 1
bash tools/gpu_round.sh r03q
