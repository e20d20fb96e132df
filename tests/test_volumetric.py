"""VolumetricDisc: oracle against the reference's own tests,
host scene loading, and the host-side constants the device kernels consume (CPU only).

The reference tests transcribed here are volumetric_disc.rs:693-786.  The Perlin noise
comes from the `noise` crate 0.9.0, which is not vendored (Cargo.lock pins noise 0.9.0,
rand 0.8.7, rand_xorshift 0.3.0): its values are restated from the crates' published
algorithms and are "parity unpinned" -- no reference test or fixture fixes them.  The
product's permutation table (host C++) and the oracle's (a separate restatement) are
checked against each other and against the structural properties of the algorithm.
"""
import ctypes as C
import math

import numpy as np
import pytest

from conftest import RESOURCES, SCENES, c2_opts, host_scene
from gr_raytracer_amd import _lib as L

VOLUMETRIC = sorted(p.name for p in SCENES.glob("*volumetric*.toml"))


def reference_disc(grt, fixed_color=None):
    """create_disc() of volumetric_disc.rs:666-691 (or the FixedTextureMap variant of
    :740-759), in flat space with the DummyTemperatureComputer (1000 K)."""
    b = grt.SceneBuilder(0)
    b.integration(100, 100.0, 0.01, 1e-5)
    b.camera((0.0, 10.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0), math.pi / 4, 8, 8)
    b.celestial(grt.Checker(0.0, 10.0, 10.0, (0, 0, 0), (0, 0, 0)))
    tex = grt.Checker(0.0 if fixed_color else 3.0, 5.0, 5.0, (255, 0, 0), (0, 0, 255))
    b.add_volumetric_disc(1.0, 3.0, tex, 1000.0, constant_temperature=True, axis=(0.0, 0.0, 1.0), num_octaves=4,
                          perlin_seed=42, max_steps=500, step_size=0.01, thickness=0.5, density_multiplier=10.0,
                          brightness_reference_temperature=1000.0, absorption=0.2, scattering=0.2,
                          noise_scale=(1.0, 1.0, 1.0), noise_offset=1.0)
    d = b.build()
    if fixed_color:  # FixedTextureMap: a checker with one colour and no beaming
        t = d.objects[0].texture
        for k in range(4):
            t.c1[k] = t.c2[k] = fixed_color[k]
    return d


def test_intersection_exists(grt, oracle):  # volumetric_disc.rs:693-700
    d = reference_disc(grt)
    hit, _, t = oracle.object_intersects(d, 0, [0.0, 0.5, 0.0, 0.0], [0.0, 1.5, 0.0, 0.0])
    assert hit and 0.0 < t <= 1.0


def test_intersection_miss_above_caps(grt, oracle):  # :702-709
    d = reference_disc(grt)
    hit, _, _ = oracle.object_intersects(d, 0, [0.0, 1.5, 0.0, 2.0], [0.0, 2.5, 0.0, 2.0])
    assert not hit


def test_density_inside_and_outside(grt, oracle):  # :711-722
    d = reference_disc(grt)
    assert oracle.vdisc_density(d, 0, [2.0, 0.0, 0.0]) > 0.0
    assert oracle.vdisc_density(d, 0, [0.2, 0.0, 0.0]) == 0.0
    assert oracle.vdisc_density(d, 0, [2.0, 0.0, 2.0]) == 0.0


def test_raymarch_produces_opacity(grt, oracle):  # :724-736
    d = reference_disc(grt)
    err, c, n = oracle.vdisc_raymarch(d, 0, [2.0, 0.0, 0.0], [1.0, 0.0, 0.0], (1.0, 1.0, 0.0))
    assert err == 0 and 0.0 < c[3] <= 1.0
    assert 0 < n <= 500


def test_raymarch_cached_exit_matches_legacy(grt, oracle):  # :738-786
    d = reference_disc(grt, fixed_color=(2.0, 1.0, 0.5, 0.7))
    e1, cached, _ = oracle.vdisc_raymarch(d, 0, [2.0, 0.0, 0.0], [1.0, 0.0, 0.0], (1.0, 1.0, 0.0), cached=True)
    e2, legacy, _ = oracle.vdisc_raymarch(d, 0, [2.0, 0.0, 0.0], [1.0, 0.0, 0.0], (1.0, 1.0, 0.0), cached=False)
    assert e1 == 0 and e2 == 0
    assert np.all(np.abs(cached - legacy) <= 1e-10), (cached, legacy)


# ---------------------------------------------------------------- Perlin (noise 0.9) --
@pytest.mark.parametrize("seed", [0, 1, 42, 0xFFFFFFFF])
def test_permutation_table_host_equals_oracle(grt, oracle, seed):
    host = np.zeros(256, np.uint8)
    grt.lib().grt_perlin_permutation(seed, host.ctypes.data_as(C.POINTER(C.c_uint8)))
    orc = oracle.perlin_table(seed)
    assert np.array_equal(host, orc)
    assert sorted(host.tolist()) == list(range(256))  # a permutation of 0..=255
    assert not np.array_equal(host, np.arange(256))


def test_perlin_structure(oracle):
    """perlin_3d: 0 on the integer lattice (every gradient is dotted with a zero
    distance), within [-1, 1], continuous across cell faces, and seed-dependent."""
    rng = np.random.default_rng(5)
    for p in rng.integers(-300, 300, size=(50, 3)):
        assert oracle.perlin(1, *map(float, p)) == 0.0
    vals = [oracle.perlin(1, *p) for p in rng.uniform(-50, 50, size=(2000, 3))]
    assert max(abs(v) for v in vals) <= 1.0 and np.std(vals) > 0.05
    for x in (3.0, -7.0):  # continuity across x = integer
        a, b = oracle.perlin(7, x - 1e-9, 0.3, 0.6), oracle.perlin(7, x + 1e-9, 0.3, 0.6)
        assert abs(a - b) < 1e-7
    assert oracle.perlin(1, 0.3, 0.4, 0.5) != oracle.perlin(2, 0.3, 0.4, 0.5)


def test_volumetric_frame(grt):
    """VolumetricDisc::new's axis / e1 / e2 (volumetric_disc.rs:61-73)."""
    def frame(ax):
        a, e1, e2 = np.zeros(3), np.zeros(3), np.zeros(3)
        grt.lib().grt_volumetric_frame(L.dptr(np.asarray(ax, float)), L.dptr(a), L.dptr(e1), L.dptr(e2))
        return a, e1, e2
    a, e1, e2 = frame((0.0, 0.0, 1.0))
    assert np.array_equal(a, [0, 0, 1]) and np.array_equal(e1, [0, -1, 0]) and np.array_equal(e2, [1, 0, 0])
    a, e1, e2 = frame((0.0, 0.0, 0.0))  # |axis|^2 <= EPSILON -> (0, 0, 1)
    assert np.array_equal(a, [0, 0, 1])
    a, e1, e2 = frame((2.0, 0.5, 0.1))  # |x| > 0.9 picks (0, 1, 0)
    assert abs(np.linalg.norm(a) - 1) < 1e-15 and abs(a @ e1) < 1e-15 and abs(a @ e2) < 1e-15


# -------------------------------------------------------------------- host loader --
@pytest.mark.parametrize("toml", VOLUMETRIC)
def test_volumetric_scenes_load(grt, toml):
    hs = host_scene(grt, toml, c2_opts(grt, width=64, height=64))
    d = hs.desc
    assert d.n_objects == 1
    o = d.objects[0]
    assert o.kind == L.OBJ_VOLUMETRIC_DISC
    assert o.num_octaves == 8 and o.march_max_steps == 50000 and o.perlin_seed == 1
    assert tuple(o.axis) == (0.0, 0.0, 1.0) and o.outer_radius > o.inner_radius > 0
    assert o.texture.kind == L.TEX_BLACKBODY and d.bb_n == 1000
    assert o.temp_kind == L.TEMP_KERR_LUT and o.lut_n == 1000


BASE = (SCENES / "schwarzschild-volumetric-stony.toml").read_text()


@pytest.mark.parametrize("mutation,needle", [  # cli/shared.rs:238-284
    (lambda s: s.replace("outer_radius = 11.0", "outer_radius = 4.0"), "outer_radius > inner_radius"),
    (lambda s: s.replace("thickness = 0.2", "thickness = 0.0"), "thickness > 0"),
    (lambda s: s.replace("max_steps = 50000", "max_steps = 0"), "max_steps > 0"),
    (lambda s: s.replace("step_size = 0.002", "step_size = -0.1"), "step_size > 0"),
    (lambda s: s.replace("brightness_reference_temperature = 900.0", "brightness_reference_temperature = 0.0"),
     "brightness_reference_temperature > 0"),
    (lambda s: s.replace("absorption = 0.4", "absorption = -1.0"), "absorption >= 0"),
    (lambda s: s.replace("scattering = 0.2", "scattering = -0.5"), "scattering >= 0"),
    (lambda s: s.replace("num_octaves = 8", "num_octaves = 8.5"), "num_octaves"),
])
def test_invalid_volumetric_configs_are_rejected(grt, tmp_path, mutation, needle):
    p = tmp_path / "scene.toml"
    p.write_text(mutation(BASE))
    with pytest.raises(grt.GrtError) as e:
        grt.HostScene(str(p), c2_opts(grt), str(RESOURCES))
    assert needle in str(e.value), str(e.value)


def test_axis_and_seed_are_read(grt, tmp_path):
    text = BASE.replace("num_octaves = 8", "num_octaves = 8\naxis = [0.0, 1.0, 1.0]\nperlin_seed = 7")
    p = tmp_path / "scene.toml"
    p.write_text(text)
    hs = grt.HostScene(str(p), c2_opts(grt), str(RESOURCES))
    o = hs.desc.objects[0]
    assert tuple(o.axis) == (0.0, 1.0, 1.0) and o.perlin_seed == 7
