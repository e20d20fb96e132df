#!/bin/bash
# March-kernel A/B of experimental builds (variants/<V>/libgrt.so), run under gpurun from the
# repo root: for each variant in the order given (repeat names to alternate), the
# VolumetricDisc frames of tools/vol_time.py (frame md5s) under rocprofv3 --kernel-trace
# --stats, and one summary line per variant with every march_kernel's mean duration.
# Usage: tools/gpu_vol_ab.sh <tag> "<scene.toml ...>" V1 V2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=$1; SCENES=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
i=0
for v in "$@"; do
  i=$((i + 1))
  d=$O/vol_${i}_$v
  GRT_LIB=$PWD/variants/$v/libgrt.so GRT_LIB_ALLOW_MISSING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $d -o run -- python3 -u tools/vol_time.py 1500 $SCENES > $d.jsonl 2> $d.err \
    || { tail -20 $d.err >&2; exit 1; }
  python3 - "$v" "$d" >> $O/vol_ab.jsonl <<'EOF' || exit 1
import csv, json, sys
v, d = sys.argv[1], sys.argv[2]
march = {}
for row in csv.DictReader(open(f"{d}/run_kernel_stats.csv")):
    if "march_kernel" in row["Name"]:
        march[row["Name"].split("(")[0].replace("void grt::", "")] = {
            "calls": int(row["Calls"]), "mean_ms": round(float(row["AverageNs"]) * 1e-6, 2),
            "min_ms": round(float(row["MinNs"]) * 1e-6, 2)}
frames = [json.loads(l) for l in open(f"{d}.jsonl") if l.startswith("{")]
print(json.dumps({"variant": v, "march": march,
                  "frames": [{k: f.get(k) for k in ("scene", "kernel_ms", "md5")} for f in frames]}))
EOF
  tail -1 $O/vol_ab.jsonl >&2
done
