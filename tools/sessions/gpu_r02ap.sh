#!/bin/bash
# r02ap: bench.py --workload c4 at full size on the final round-2 build on one GPU (the north-star frame, 4096^2
# kerr.toml, one rank: the strong-scaling base point), with a heartbeat file while it runs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02ap
mkdir -p "$OUT"
( while true; do date +%s >> "$OUT/heartbeat"; sleep 50; done ) &
HB=$!
timeout -k 10 900 python3 bench.py --workload c4 --steps 1 --warmup 0 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
rc=$?
kill $HB
[ $rc -ne 0 ] && { tail -20 "$OUT/bench_c4.err" >&2; exit $rc; }
cat "$OUT/bench_c4.json" >&2
