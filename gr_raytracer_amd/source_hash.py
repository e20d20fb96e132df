"""SHA-256 of the sources libgrt.so is built from.

The Makefile stamps this hash into the library (`grt_source_hash()`, generated at build
time), and `_lib.lib()` refuses a library whose stamp differs from the checkout it is
loaded from, so a stale prebuilt `.so` cannot pass for the current sources.

Hashed: every file under gr_raytracer_amd/csrc/{device,host,cli} and the Makefile, and
include/*.h -- as "<sha256 of the file>  <path relative to the repo root>" lines,
sorted by path, then the SHA-256 of those lines.  Run as a script it prints the hash
(the Makefile's call).
"""
from __future__ import annotations

import hashlib
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SUFFIXES = {".hip", ".h", ".cpp", ".inc"}


def source_files(root: Path = ROOT) -> list:
    csrc = root / "gr_raytracer_amd" / "csrc"
    files = [csrc / "Makefile"]
    for sub in ("device", "host", "cli"):
        files += [p for p in (csrc / sub).iterdir() if p.suffix in SUFFIXES]
    files += [p for p in (root / "include").iterdir() if p.suffix == ".h"]
    return sorted(files, key=lambda p: p.relative_to(root).as_posix())


def source_hash(root: Path = ROOT) -> str:
    lines = []
    for p in source_files(root):
        lines.append(f"{hashlib.sha256(p.read_bytes()).hexdigest()}  {p.relative_to(root).as_posix()}\n")
    return hashlib.sha256("".join(lines).encode()).hexdigest()


if __name__ == "__main__":
    print(source_hash(Path(sys.argv[1]).resolve() if len(sys.argv) > 1 else ROOT))
