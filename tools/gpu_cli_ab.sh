#!/bin/bash
# Process wall-clock A/B of grt CLI builds (variants/<V>/grt with its libgrt.so), C2 at
# 1 spp, alternating in the order given; one JSON line per run with the CLI's phases.
# Usage (gpurun, repo root): tools/gpu_cli_ab.sh <tag> V1 V2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; shift; mkdir -p $O
T=$(mktemp -d); printf '\n[adaptive_sampling]\nenabled = false\n' | cat tests/golden/scenes/schwarzschild.toml - > $T/c2.toml
A="--width=1500 --height=1500 --camera-position=-16.0,0.0,3.5 --theta=-3.142 --psi=0.0 --phi=0.0 --max-steps=100000 --resource-root tests/golden --config-file $T/c2.toml render --filename $T/c2.png"
export GRT_LIB_ALLOW_MISSING=1
for v in "$@"; do
  t0=$EPOCHREALTIME
  timeout -k 10 120 variants/$v/grt $A > $O/cli_$v.log 2>&1 || { tail $O/cli_$v.log >&2; exit 1; }
  t1=$EPOCHREALTIME
  python3 - "$v" "$t0" "$t1" "$O/cli_$v.log" >> $O/cli_ab.jsonl <<'PY'
import json, re, sys
v, t0, t1, log = sys.argv[1], float(sys.argv[2]), float(sys.argv[3]), sys.argv[4]
ph = re.search(r"phases \(ms\): (.*)", open(log).read()).group(1)
print(json.dumps({"variant": v, "process_wall_s": round(t1 - t0, 3), "phases": ph}))
PY
  tail -1 $O/cli_ab.jsonl >&2
done
