"""`blackbody` and `blackbody-spectrum` subcommands (cli/blackbody.rs, SURVEY.md 8(f)
row 4), host-only in the reference and here (CPU tests).

run_blackbody prints integrate_blackbody_xyz(T, z) and its untone-mapped sRGB
(xyz_to_srgb, color.rs:225-241); the reference's own KATs pin that pair
(black_body_radiation.rs:63-73: 1000 K -> (255, 60, 0), 10000 K -> (137, 146, 172) at
exposure 1/(X+Y+Z)).  run_blackbody_spectrum maps a T x z grid through the output
stage; its pixels must be the oracle's output stage applied to the same XYZ grid.
"""
import math
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from test_oracle_kats import xyz_to_srgb
from test_trajectory import rust_display

GRT = ROOT / "gr_raytracer_amd" / "lib" / "grt"


@pytest.mark.parametrize("temperature,rgb", [(1000.0, (255, 60, 0)), (10000.0, (137, 146, 172))])
def test_host_xyz_to_srgb_reference_kats(grt, temperature, rgb):
    from gr_raytracer_amd import _lib as L

    c = np.ascontiguousarray(grt.blackbody_xyz(temperature, 1.0))
    out = np.zeros(3, np.uint8)
    L.lib().grt_xyz_to_srgb(L.dptr(c), 1.0 / (c[0] + c[1] + c[2]), L.ptr(out, L.C.c_uint8))
    assert tuple(int(v) for v in out) == rgb


@pytest.mark.parametrize("temperature,redshift", [(1000.0, 1.0), (6500.0, 0.7), (10000.0, 1.5), (2.5e4, 2.0)])
def test_blackbody_subcommand_output(grt, temperature, redshift):
    r = subprocess.run([str(GRT), "blackbody", "-t", repr(temperature), "-r", repr(redshift)], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    xyz = grt.blackbody_xyz(temperature, redshift)
    c = xyz_to_srgb(xyz, 1.0)
    want = [f"Blackbody color at T={rust_display(temperature)}K (redshift={rust_display(redshift)}):",
            f"XYZ:  {xyz[0]:.4f}, {xyz[1]:.4f}, {xyz[2]:.4f}",
            f"sRGB: R={c[0]}, G={c[1]}, B={c[2]}",
            f"sRGB: R={c[0] / 255.0:.4f}, G={c[1] / 255.0:.4f}, B={c[2] / 255.0:.4f}",
            f"Color block: \x1b[48;2;{c[0]};{c[1]};{c[2]}m      \x1b[0m"]
    assert r.stdout.split("\n")[:5] == want


@pytest.mark.parametrize("tone,tone_id", [("reinhard", 0), ("global-linear", 1)])
def test_blackbody_spectrum_image(grt, oracle, tmp_path, tone, tone_id):
    Image = pytest.importorskip("PIL.Image")
    w, h = 23, 9
    args = dict(min_temperature=1500.0, max_temperature=12000.0, min_redshift=0.6, max_redshift=1.8)
    png = tmp_path / "spectrum.png"
    r = subprocess.run([str(GRT), f"--tone-mapping={tone}", "blackbody-spectrum", "--width", str(w), "--height",
                        str(h), *sum(([f"--{k.replace('_', '-')}", repr(v)] for k, v in args.items()), []),
                        "-f", str(png)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    img = np.asarray(Image.open(png))
    assert img.shape == (h, w, 4) and np.all(img[..., 3] == 255)
    xyza = np.zeros((w * h, 4))
    for i in range(w * h):  # cli/blackbody.rs:63-70
        x, y = float(i % w), float(i // w)
        t = args["min_temperature"] + x * (args["max_temperature"] - args["min_temperature"]) / (w - 1.0)
        z = args["min_redshift"] + y * (args["max_redshift"] - args["min_redshift"]) / (h - 1.0)
        xyza[i, :3] = grt.blackbody_xyz(t, z)
        xyza[i, 3] = 1.0
    want = oracle.xyz_to_srgb8(xyza, tone_id).reshape(h, w, 3)
    assert np.array_equal(img[..., :3], want)
    assert not math.isnan(float(img.mean()))
