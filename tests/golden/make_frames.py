"""Generate the committed golden frame fixtures (tests/golden/frames/*.npz).

Each fixture is a crop of one BASELINE / scene-definitions configuration rendered by the
ORACLE (oracle/, the reference algorithm restated on the CPU, itself pinned by the
reference's known-answer tests in tests/test_oracle_kats.py and tests/test_volumetric.py).
The Rust reference cannot be built here, so these frames pin the build
against its own checker, not against the Rust binary: a change of the oracle, the host
scene setup or glibc shows up as a fixture mismatch (tests/test_golden_frames.py), and
the GPU is compared with the frozen values.

usage: python tests/golden/make_frames.py   (rewrites tests/golden/frames/)
"""
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]

import numpy as np  # noqa: E402

# name: (scene toml, options, crop (row0, col0, rows, cols))
C2 = dict(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
C3 = dict(width=1500, height=1500, camera_position=(-10.0, 0.0, -0.5), theta=-3.14159, max_steps=1000000)
C4 = dict(width=4096, height=4096, camera_position=(-10.0, 0.0, -0.5), theta=1.52, psi=-1.57, max_steps=1000000)
FRAMES = {
    "c1_euclidean": ("euclidean.toml", dict(width=256, height=256), (100, 100, 40, 48)),
    "c2_shadow_edge": ("schwarzschild.toml", C2, (680, 600, 24, 48)),
    "c2_disc": ("schwarzschild.toml", C2, (795, 540, 24, 40)),
    "c3_kerr_bl": ("kerr-bl.toml", C3, (700, 300, 24, 32)),
    "c4_kerr_schild": ("kerr.toml", C4, (2900, 1200, 12, 16)),
    "vol_schwarzschild_stony": ("schwarzschild-volumetric-stony.toml", dict(C2, width=160, height=160),
                                (56, 40, 16, 24)),
    "vol_kerr_bl_streaky": ("kerr-bl-volumetric-streaky.toml", dict(C3, width=160, height=160), (76, 20, 12, 32)),
}


def main():
    import gr_raytracer_amd as g
    import pyoracle as O
    from conftest import RESOURCES, SCENES

    out = HERE / "frames"
    out.mkdir(exist_ok=True)
    manifest = {}
    for name, (toml, opts, rect) in FRAMES.items():
        hs = g.HostScene(str(SCENES / toml), g.GlobalOpts(**opts), str(RESOURCES))
        r = O.render_pixels(hs.desc, *rect, threads=8)
        np.savez_compressed(out / f"{name}.npz", xyza64=r["xyza"], ray_class=r["ray_class"], status=r["status"],
                            stop=r["stop"], steps=r["steps"])
        manifest[name] = {"scene": toml, "opts": opts, "rect": list(rect)}
        print(name, rect, "accepted", r["accepted"], "classes", np.bincount(r["ray_class"], minlength=3).tolist(),
              f"{r['wall_s']:.1f} s", flush=True)
    (out / "manifest.json").write_text(json.dumps(manifest, indent=1) + "\n")


if __name__ == "__main__":
    main()
