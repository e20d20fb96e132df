"""Host side of the boundary on CPU: TOML scene loading (configuration.rs schema),
texture decoding, camera tetrads, LUT builders and input validation."""
import ctypes as C
import math

import numpy as np
import pytest

from conftest import RESOURCES, SCENES, c1_opts, c2_opts, c3_opts, c4_opts, host_scene

SCENE_OPTS = {"euclidean.toml": c1_opts, "schwarzschild.toml": c2_opts, "schwarzschild-sphere.toml": c2_opts,
              "kerr.toml": c4_opts, "kerr-sphere.toml": c4_opts, "kerr-bl.toml": c3_opts,
              "euclidean-spherical.toml": c1_opts}
GEOMETRY = {"euclidean.toml": 0, "schwarzschild.toml": 1, "schwarzschild-sphere.toml": 1, "kerr.toml": 2,
            "kerr-sphere.toml": 2, "kerr-bl.toml": 3, "euclidean-spherical.toml": 4}


@pytest.mark.parametrize("name", sorted(SCENE_OPTS))
def test_vendored_scenes_load(grt, name):
    hs = host_scene(grt, name, SCENE_OPTS[name](grt))
    d = hs.desc
    assert d.geometry == GEOMETRY[name]
    assert 1 <= d.n_objects <= 8
    assert d.camera.rows > 0 and d.camera.cols > 0
    assert abs(d.camera.alpha - math.pi / 4) < 1e-15  # Camera::new default (cli/shared.rs)


def _minkowski_check(oracle, d):
    """g(e_a, e_b) = eta_ab * signature (TetradValidator, tetrad.rs:60-131)."""
    pos = list(d.camera.position)
    tet = [list(d.camera.tetrad[i]) for i in range(4)]
    g = np.array([[oracle.inner_product(d, pos, tet[i], tet[j]) for j in range(4)] for i in range(4)])
    off = g - np.diag(np.diag(g))
    assert np.max(np.abs(off)) < 1e-9, g
    assert np.allclose(np.abs(np.diag(g)), 1.0, atol=1e-9), g
    assert np.sign(g[0, 0]) == -np.sign(g[1, 1]) == -np.sign(g[2, 2]) == -np.sign(g[3, 3])


@pytest.mark.parametrize("name", ["schwarzschild.toml", "kerr.toml", "kerr-bl.toml", "euclidean.toml",
                                  "euclidean-spherical.toml"])
def test_camera_tetrads_are_orthonormal(grt, oracle, name):
    hs = host_scene(grt, name, SCENE_OPTS[name](grt))
    _minkowski_check(oracle, hs.desc)


def test_bitmap_textures_decode_like_pil(grt):
    Image = pytest.importorskip("PIL.Image")
    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt))
    d = hs.desc
    textures = [("celestial.png", d.celestial)] + [(n, d.objects[i].texture)
                                                   for i, n in enumerate(["disk.png", "sphere.png"])]
    for fname, t in textures:
        want = np.asarray(Image.open(RESOURCES / "resources" / fname).convert("RGBA"))
        assert (t.height, t.width) == want.shape[:2]
        got = np.ctypeslib.as_array(C.cast(t.rgba, C.POINTER(C.c_uint8)), shape=(t.height, t.width, 4))
        assert np.array_equal(got, want), fname


def _write_scene(tmp_path, text):
    p = tmp_path / "scene.toml"
    p.write_text(text)
    return p


BASE = (SCENES / "schwarzschild.toml").read_text()


@pytest.mark.parametrize("mutation,needle", [
    (lambda s: s.replace("[geometry_type.Schwarzschild]", "[geometry_type.Minkowski]"), "geometry"),
    (lambda s: s + "\n[adaptive_sampling]\nenabled = true\nsamples_per_axis = 0\n", "samples_per_axis"),
    (lambda s: s + "\n[adaptive_sampling]\nluminance_contrast_threshold = 1.5\n", "luminance_contrast_threshold"),
    (lambda s: s.replace('path = "resources/disk.png"', 'path = "resources/missing.png"'), "missing.png"),
    (lambda s: s.replace("inner_radius = 3.0", "inner_radius = 3.0 3.0"), "TOML"),
    (lambda s: s.replace("objects.Sphere", "objects.VolumetricDisc"), "inner_radius"),
])
def test_invalid_scenes_are_rejected(grt, tmp_path, mutation, needle):
    p = _write_scene(tmp_path, mutation(BASE))
    with pytest.raises(grt.GrtError) as e:
        grt.HostScene(str(p), c2_opts(grt), str(RESOURCES))
    assert needle in str(e.value), str(e.value)


def test_past_directed_camera_velocity_is_rejected(grt, tmp_path):
    text = BASE + '\n[camera_velocity.Explicit]\ncomponents = [-1.0, 0.0, 0.0, 0.0]\n'
    p = _write_scene(tmp_path, text)
    with pytest.raises(grt.GrtError):
        grt.HostScene(str(p), c2_opts(grt, camera_position=(-16.0, 0.0, 0.0)), str(RESOURCES))


def test_adaptive_defaults_follow_the_reference(grt):
    """Stock TOMLs supersample 4x4 by default (configuration.rs AdaptiveSamplingConfig)."""
    hs = host_scene(grt, "euclidean.toml", c1_opts(grt))
    ad = hs.adaptive
    assert ad.enabled == 1 and ad.samples_per_axis == 4


def test_kerr_temperature_lut_is_monotone_in_radius(grt):
    lr, lt, ri = grt.kerr_temperature_lut(2000.0, 15.0, 0.499, 1.0)
    assert len(lr) == 1000 and np.all(np.diff(lr) > 0)
    assert abs(lr[0] - ri) < 1e-12 and ri == grt.r_isco(1.0, 0.499)
    assert np.all(np.isfinite(lt)) and lt.max() > 0
