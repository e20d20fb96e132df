"""Committed golden frames (tests/golden/frames/, written by tests/golden/make_frames.py).

Crops of C1-C4 and of two VolumetricDisc scenes, rendered once by the oracle and frozen.
They pin the build against its own checker (the Rust reference cannot be built here,
SURVEY.md 8(c)): the CPU test catches any drift of the oracle, the host scene setup or
the libm; the GPU test holds the device to the frozen values with the north-star bar
(1e-4 relative per channel, identical class / status / stop reason).
"""
import json

import numpy as np
import pytest

from conftest import RESOURCES, SCENES

GOLDEN = SCENES.parent / "frames"
MANIFEST = json.loads((GOLDEN / "manifest.json").read_text())


def load(name):
    z = np.load(GOLDEN / f"{name}.npz")
    return {k: z[k] for k in z.files}


def host_scene(grt, name):
    m = MANIFEST[name]
    return grt.HostScene(str(SCENES / m["scene"]), grt.GlobalOpts(**m["opts"]), str(RESOURCES)), tuple(m["rect"])


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_oracle_reproduces_golden_frame(grt, oracle, name):
    hs, rect = host_scene(grt, name)
    want = load(name)
    got = oracle.render_pixels(hs.desc, *rect, threads=8)
    assert np.array_equal(got["xyza"], want["xyza64"])
    for k in ("ray_class", "status", "stop", "steps"):
        assert np.array_equal(got[k], want[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_gpu_matches_golden_frame(grt, gpu, name):
    hs, rect = host_scene(grt, name)
    want = load(name)
    sc = grt.Scene(hs.desc_ptr(), keepalive=hs, adaptive=hs.adaptive)
    got = sc.render_pixels(*rect)
    ref = want["xyza64"]
    ok = np.all(np.abs(got.xyza64 - ref) <= 1e-4 * np.maximum(np.abs(ref), 1e-6), axis=1)
    assert ok.all(), (name, np.where(~ok)[0][:8])
    assert np.array_equal(got.ray_class, want["ray_class"])
    assert np.array_equal(got.status, want["status"])
    assert np.array_equal(got.stop_reason, want["stop"])
    assert np.mean(got.steps == want["steps"]) >= 0.99
    exact = np.mean(np.all(got.xyza64 == ref, axis=1))
    print(f"{name}: {exact:.3f} of the pixels bit-identical to the frozen oracle frame")
