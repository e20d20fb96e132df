#!/bin/bash
# isa_stats.sh [EXTRA_HIPFLAGS...]: register / spill / code-size summary of the integrate kernels
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
W=$(mktemp -d /tmp/isa.XXXX); cd $W
/opt/rocm/bin/hipcc -I$ROOT/include --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -munsafe-fp-atomics --save-temps "$@" -c ${SRC:-$ROOT/gr_raytracer_amd/csrc/device/geodesic.hip} -o g.o 2>/dev/null
B=$(basename ${SRC:-geodesic.hip} .hip); S=$B-hip-amdgcn-amd-amdhsa-gfx950.s
python3 - "$S" $B-hip-amdgcn-amd-amdhsa-gfx950.out <<'PY'
import re, subprocess, sys
s = open(sys.argv[1]).read()
syms = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-s", "--wide", sys.argv[2]], capture_output=True, text=True).stdout
size = {l.split()[7]: int(l.split()[2]) for l in syms.splitlines() if ("integrate_kernel" in l or "tail_kernel" in l) and "FUNC" in l}
for m in re.finditer(r"\.name:\s+(_ZN3grt16integrate_kernelILi(\d)\S*)", s):
    pass
for md in re.split(r"\n  - ", s.split("amdhsa.kernels:")[1]):
    name = re.search(r"\.name:\s+(\S+)", md)
    if not name or ("integrate_kernel" not in name.group(1) and "tail_kernel" not in name.group(1)): continue
    g = lambda k: re.search(r"\.%s:\s+(\d+)" % k, md).group(1)
    n = name.group(1)
    kind = 'tail' if 'tail_kernel' in n else 'integrate'
    print(f"{kind}<{n.split('ILi')[1][0]}> vgpr {g('vgpr_count')} agpr {g('agpr_count')} "
          f"vspill {g('vgpr_spill_count')} sgpr {g('sgpr_count')} sspill {g('sgpr_spill_count')} code {size.get(n)}")
PY
rm -rf $W
