"""VolumetricDisc on the GPU vs the oracle (marker `gpu`).

The device path: integrate_kernel<G, true> records each window-nearest capture-region
crossing with its chord direction, shade_kernel<G, 1> gathers the raymarch jobs,
march_kernel<G> raymarches them (lane refill), shade_kernel<G, 2> composites.  The
oracle runs the reference's algorithm literally (whole trajectory, post-hoc window
pass, raymarch inside Objects::intersects).  Bar: tests/test_gpu_parity.check_parity
(1e-4 per channel, identical class / status / stop).

Parity of the Perlin noise itself against the Rust `noise` 0.9.0 crate is unpinned
(not vendored); GPU and oracle share the restated algorithm, the oracle's part of it
is pinned by the reference's volumetric_disc.rs tests (tests/test_volumetric.py).
"""
import numpy as np
import pytest

from conftest import RESOURCES, SCENES, c2_opts, c3_opts, c4_opts
from test_gpu_parity import check_parity, gpu_scene, oracle_pair

pytestmark = pytest.mark.gpu


def vol_host_scene(grt, toml, width, height=None, path=None):
    # the reference's example cameras: C2's (Schwarzschild), C3's (KerrBL), C4's (Kerr-Schild)
    mk = c4_opts if toml.startswith("kerr-volumetric") else (c3_opts if toml.startswith("kerr") else c2_opts)
    opts = mk(grt, width=width, height=height or width)
    return grt.HostScene(str(path or (SCENES / toml)), opts, str(RESOURCES))


def compare(grt, oracle, hs, rect, max_sensitive=0.02):
    sc = gpu_scene(grt, hs)
    got = sc.render_pixels(*rect)
    ref, probes = oracle_pair(oracle, hs.desc, *rect)
    check_parity(got, ref, probes, max_sensitive=max_sensitive)
    return got, ref


# 160 x 160 frames (C2 / C3 cameras); crops through the gas, its inner edge and the shadow
CROPS = [
    ("schwarzschild-volumetric-stony.toml", (52, 36, 24, 32)),
    ("schwarzschild-volumetric-streaky.toml", (84, 16, 16, 40)),
    ("schwarzschild-volumetric-dense.toml", (60, 56, 20, 48)),
    ("kerr-bl-volumetric-stony.toml", (70, 40, 20, 40)),
    ("kerr-bl-volumetric-streaky.toml", (74, 20, 16, 40)),
]


@pytest.mark.parametrize("toml,rect", CROPS)
def test_volumetric_scene_crops(grt, oracle, gpu, toml, rect):
    hs = vol_host_scene(grt, toml, 160)
    got, ref = compare(grt, oracle, hs, rect)
    assert got.stats["march_jobs"] > 0 and got.stats["march_samples"] >= got.stats["march_jobs"]
    assert np.any(got.ray_class == 2)  # the gas is opaque enough to classify pixels as hits


def test_kerr_schild_volumetric_crop(grt, oracle, gpu):
    """kerr-volumetric-stony.toml (Kerr-Schild chart, Cartesian: no far-field filter).

    Here the oracle's own last-ulp probes move most pixels (measured: 185 of 240): the
    finite-difference metric derivatives make the step controller's accept / reject
    decisions sensitive to the last ulp, a changed step sequence moves the window chord
    that crosses the gas's capture boundary, and the fBm (up to 512 x 25 cycles per unit)
    turns that shift into a different colour.  The GPU integrates Kerr-Schild bit for bit
    like the oracle (glibc-exact pow; no trig on this chart), so it is held to the oracle
    itself: 95% of the pixels within 1e-4 with identical class."""
    from test_gpu_parity import agree

    hs = vol_host_scene(grt, "kerr-volumetric-stony.toml", 160)
    rect = (76, 0, 6, 40)
    got = gpu_scene(grt, hs).render_pixels(*rect)
    ref = oracle.render_pixels(hs.desc, *rect, threads=16)
    ok = agree(got.xyza64, got.ray_class, ref)
    assert ok.mean() >= 0.95, (ok.mean(), np.where(~ok)[0][:10])
    assert np.array_equal(got.status, ref["status"]) and np.mean(got.steps == ref["steps"]) >= 0.95
    assert got.stats["march_jobs"] > 0 and np.any(got.ray_class == 2)


FLAT = """celestial_temperature = 0.0

[celestial_texture.Bitmap]
beaming_exponent = 0.0
path = "resources/celestial.png"

[geometry_type]
Euclidean = {}

[[objects]]

[objects.VolumetricDisc]
inner_radius = 2.0
outer_radius = 9.0
temperature = 3000.0
axis = [0.1, 0.2, 1.0]
num_octaves = 6
perlin_seed = 11
max_steps = 4000
step_size = 0.01
thickness = 0.4
density_multiplier = 40.0
brightness_reference_temperature = 2000.0
absorption = 0.5
scattering = 0.5
noise_scale = [3.0, 2.0, 4.0]
noise_offset = 0.1

[objects.VolumetricDisc.texture.Checker]
beaming_exponent = 1.0
width = 12.0
height = 12.0
color1 = [255, 200, 120]
color2 = [40, 60, 200]
"""


def test_flat_space_tilted_gas_full_frame(grt, oracle, gpu, tmp_path):
    """Euclidean geometry (straight rays, cheap integration, constant temperature) with a
    tilted axis and a checker texture: the raymarch, the general-axis capture region and
    the texture path over a whole 96 x 96 frame."""
    p = tmp_path / "flat-volumetric.toml"
    p.write_text(FLAT)
    hs = grt.HostScene(str(p), grt.GlobalOpts(width=96, height=96), str(RESOURCES))
    got, ref = compare(grt, oracle, hs, (0, 0, 96, 96))
    assert got.stats["march_jobs"] > 500
    assert np.any(got.ray_class == 2) and np.any(got.ray_class == 0)


def test_volumetric_row_shards_equal_the_frame(grt, gpu):
    """Cyclic row-band shards of a volumetric frame are bit-identical to one launch."""
    hs = vol_host_scene(grt, "schwarzschild-volumetric-stony.toml", 96)
    sc = gpu_scene(grt, hs)
    full = sc.render_pixels(0, 0, 96, 96)
    rows = np.arange(96)
    for s in range(3):
        part = sc.render_shard(8, s, 3)
        mine = rows[(rows // 8) % 3 == s]
        idx = (mine[:, None] * 96 + np.arange(96)[None, :]).ravel()
        assert np.array_equal(part.xyza64, full.xyza64[idx])
        assert np.array_equal(part.ray_class, full.ray_class[idx])


def test_volumetric_adaptive_section(grt, oracle, gpu):
    """The stock TOMLs supersample 4x4: the jittered sub-rays go through the same
    volumetric pipeline (offset work list)."""
    hs = vol_host_scene(grt, "schwarzschild-volumetric-streaky.toml", 64)
    sc = gpu_scene(grt, hs)
    r0, c0, r1, c1 = 26, 8, 34, 56  # gas in front of and beside the shadow
    out, cls, nsel, st = sc.render_section(r0, c0, r1, c1)
    ref, ref_cls, ref_nsel = oracle.render_section(hs.desc, r0, c0, r1, c1, hs.adaptive)
    assert nsel == ref_nsel and nsel > 0 and st["march_jobs"] > 0
    ok = np.all(np.abs(out - ref) <= 1e-4 * np.maximum(np.abs(ref), 1e-6), axis=1)
    assert ok.mean() >= 0.98, ok.mean()


def test_cli_renders_a_stock_volumetric_scene(grt, oracle, gpu, tmp_path):
    """`grt ... --config-file=schwarzschild-volumetric-stony.toml render` (stock TOML:
    adaptive 4x4 on): the raw f64 frame is grt_render_section's, the PNG its reference
    output stage."""
    import subprocess
    from pathlib import Path

    Image = pytest.importorskip("PIL.Image")
    root = Path(__file__).resolve().parents[1]
    png, raw = tmp_path / "vol.png", tmp_path / "vol.raw"
    toml = SCENES / "schwarzschild-volumetric-stony.toml"
    subprocess.run([str(root / "gr_raytracer_amd" / "lib" / "grt"), "--width=48", "--height=40",
                    "--camera-position=-16.0,0.0,3.5", "--theta=-3.142", "--max-steps=100000",
                    f"--config-file={toml}", f"--resource-root={RESOURCES}", "render", f"--filename={png}",
                    f"--raw-out={raw}", f"--device={gpu}"], check=True, timeout=300)
    x = np.fromfile(raw, np.float64).reshape(-1, 4)
    hs = grt.HostScene(str(toml), c2_opts(grt, width=48, height=40), str(RESOURCES))
    sc = gpu_scene(grt, hs)
    out, cls, nsel, st = sc.render_section()
    assert np.array_equal(x, out) and nsel > 0 and st["march_jobs"] > 0
    img = np.asarray(Image.open(png).convert("RGB")).reshape(-1, 3)
    assert np.array_equal(img, oracle.xyz_to_srgb8(x, 0))
