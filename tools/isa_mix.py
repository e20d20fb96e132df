"""Instruction mix of one straight-line RHS evaluation of an integrate kernel.

usage: python tools/isa_mix.py [geometry=1] [kernel .s from hipcc --save-temps -gline-tables-only]
Builds geodesic.hip for gfx950 with line tables (unless a .s is given), takes
integrate_kernel<geometry, false>, splits it into basic blocks and reports, for the
largest block that holds glibc sincos code and at least three IEEE reciprocals (the
wave-uniform region-B RHS of with_sincos), its instructions by category:
  division  v_div_scale/fmas/fixup_f64, v_rcp_f64 and the Newton v_fma/v_fmac_f64
  sincos    VALU attributed (.loc) to glibc_math.h
  f64       the other FP64 VALU (the reference's arithmetic)
  other     the remaining VALU (selects, integer, moves)
  salu/lds  scalar instructions (constants, branches) / LDS table reads."""
import collections
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
G = int(sys.argv[1]) if len(sys.argv) > 1 else 1
if len(sys.argv) > 2:
    asm = Path(sys.argv[2])
else:
    tmp = Path(tempfile.mkdtemp(prefix="isa_mix."))
    subprocess.run(["/opt/rocm/bin/hipcc", f"-I{ROOT}/include", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    "-ffp-contract=off", "-fno-fast-math", "-munsafe-fp-atomics", "-gline-tables-only", "--save-temps",
                    "-c", str(ROOT / "gr_raytracer_amd/csrc/device/geodesic.hip"), "-o", str(tmp / "g.o")],
                   cwd=tmp, check=True, capture_output=True)
    asm = tmp / "geodesic-hip-amdgcn-amd-amdhsa-gfx950.s"
S = asm.read_text().split("\n")
name = f"_ZN3grt16integrate_kernelILi{G}ELb0EEEvPKNS_8DevSceneENS_8WorkListENS_9WorkspaceEPyS6_NS_8TailListE"
start = next(i for i, l in enumerate(S) if l.startswith(name + ":"))
end = next(i for i in range(start, len(S)) if S[i].startswith(".Lfunc_end"))
files = {}
for l in S[:start]:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m:
        files[int(m.group(1))] = (m.group(3) or m.group(2)).split("/")[-1]
blocks, cur, loc = [], None, None
for l in S[start:end]:
    m = re.match(r"^(\.LBB\S+):", l)
    if m or cur is None:
        cur = {"name": m.group(1) if m else "entry", "ins": []}
        blocks.append(cur)
        if m:
            continue
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        loc = files.get(int(m.group(1)), "?")
        continue
    t = l.strip()
    if t and not t.startswith((";", ".")):
        cur["ins"].append((t.split()[0], loc))

DIV = ("v_div_scale_f64", "v_div_fmas_f64", "v_div_fixup_f64", "v_rcp_f64", "v_fma_f64", "v_fmac_f64")


def cat(op, loc):
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if not op.startswith("v_"):
        return "mem"
    if op.split("_e32")[0].split("_e64")[0] in DIV:
        return "division"
    if loc == "glibc_math.h":
        return "sincos"
    if "_f64" in op:
        return "f64"
    return "other"


# the RHS: sincos and at least three reciprocals (five divisions, two sharing one)
# with ALL=1: every such block (the region-B forms: table / Taylor sincos, with the IEEE
# or the range-free divisions), largest first
import os  # noqa: E402
cands = sorted((b for b in blocks if any(cat(o, l) == "sincos" for o, l in b["ins"]) and
                sum(o.startswith("v_rcp_f64") for o, _ in b["ins"]) >= 3), key=lambda b: -len(b["ins"]))
for best in (cands if os.environ.get("ALL") == "1" else cands[:1]):
    c = collections.Counter(cat(o, l) for o, l in best["ins"])
    valu = sum(v for k, v in c.items() if k in ("division", "sincos", "f64", "other"))
    print(f"integrate_kernel<{G}, false> {best['name']}: {len(best['ins'])} instructions, {valu} VALU")
    for k in ("f64", "division", "sincos", "other", "salu", "lds", "mem"):
        print(f"  {k:9s} {c.get(k, 0):4d}" + (f"  ({c.get(k, 0) / valu:.0%} of VALU)" if k in ("f64", "division", "sincos", "other") else ""))
    ops = collections.Counter(o for o, l in best["ins"] if cat(o, l) in ("division",))
    print("  division ops:", dict(ops))
