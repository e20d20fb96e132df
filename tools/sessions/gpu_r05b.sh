#!/bin/bash
# r05b: the aee1fe7 nondeterminism (C3 frame wrong with the LDS Cartesian cache + 64-B
# candidate records): C3 md5 over 3 runs of aee1fe7 (aee), aee1fe7 without the LDS cache
# (aee_nolds), this build with the LDS cache added back (head_lds) and this build (main);
# per-pixel class / stop / steps / hits saved for the comparison
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
( while sleep 60; do echo "[heartbeat] $(date +%T)" >&2; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=gpurun_out/r05b; mkdir -p $OUT
export GRT_LIB_ALLOW_MISSING=1
for v in main aee aee_nolds head_lds; do
  save=1; [ $v = aee ] && save=2; [ $v = head_lds ] && save=2
  GRT_LIB=$PWD/variants/$v/libgrt.so timeout -k 10 120 python3 -u tools/c3_det.py $OUT/$v 3 $save > $OUT/$v.jsonl 2>&1 || { cat $OUT/$v.jsonl >&2; exit 1; }
  sed "s/^/$v /" $OUT/$v.jsonl >&2
done
