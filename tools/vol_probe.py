"""Oracle preview of a volumetric scene (CPU): class map, timing, march samples.

usage: python tools/vol_probe.py <scene toml under tests/golden/scenes> <width> [rows...]
Used to pick the GPU parity crops of tests/test_gpu_volumetric.py.
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]

import numpy as np  # noqa: E402

import gr_raytracer_amd as g  # noqa: E402
import pyoracle as O  # noqa: E402
from conftest import c2_opts, c3_opts, c4_opts, host_scene  # noqa: E402


def main():
    toml, W = sys.argv[1], int(sys.argv[2])
    # C2 camera for Schwarzschild, C3's for KerrBL, C4's for Kerr-Schild (as the reference's examples)
    mk = c4_opts if toml.startswith("kerr-") and not toml.startswith("kerr-bl") else (c3_opts if "kerr" in toml else c2_opts)
    opts = mk(g, width=W, height=W)
    hs = host_scene(g, toml, opts)
    t = time.time()
    r = O.render_pixels(hs.desc, 0, 0, W, W, threads=8)
    print(toml, W, "oracle s", round(time.time() - t, 1), "accepted", r["accepted"])
    cls = r["ray_class"].reshape(W, W)
    st = r["status"].reshape(W, W)
    print("classes", np.bincount(cls.ravel(), minlength=3), "status", np.bincount(st.ravel()))
    step = max(1, W // 64)
    for row in range(0, W, max(1, W // 32)):
        print(f"{row:4d} " + "".join("#" if cls[row, c] == 2 else ("." if cls[row, c] == 0 else " ")
                                     for c in range(0, W, step)))


if __name__ == "__main__":
    main()
