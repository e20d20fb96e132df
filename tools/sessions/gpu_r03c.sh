#!/bin/bash
# r03c: bisect the C3 full-frame nondeterminism (rays left unintegrated) over builds
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03c
mkdir -p "$OUT"
for v in noappend w2; do
  GRT_LIB=$PWD/variants/$v/libgrt.so timeout -k 10 300 python3 tools/diag_frames.py c3 > "$OUT/diag_$v.jsonl" 2>&1 || { cat "$OUT/diag_$v.jsonl" >&2; exit 1; }
  echo "== $v" >&2; grep -v amdgpu.ids "$OUT/diag_$v.jsonl" >&2
done
