"""Long-ray hand-off of Kerr-Schild traces (TailList / tail_kernel).

The integrate kernel hands its remaining rays to tail_kernel once the tile queue is
drained and few rays are live; tail_kernel splits each RHS evaluation over the 4 lanes
of a quad.  Scheduling only: every output must be bit-identical to integrating each ray
on one lane (hand-off off), whatever the threshold."""
import numpy as np
import pytest

from conftest import c4_opts, host_scene


def _set_tail(grt, v):
    grt.scene.set_tail(v)


def test_set_tail_rejects_bad_thresholds(grt):
    assert grt._lib.lib().grt_set_tail(-2) != 0
    assert grt._lib.lib().grt_set_tail(-1) == 0


def _render(grt, sc, rect):
    r = sc.render_pixels(*rect)
    return r, sc.tail_handoffs()


@pytest.mark.gpu
@pytest.mark.parametrize("rect", [(1816, 2792, 24, 24), (2000, 2000, 16, 16)])
def test_tail_hand_off_is_bit_identical(grt, gpu, rect):
    """C4's camera (kerr.toml) at its longest rays and at the photon ring, max_steps 1e5:
    hand-off off, automatic, immediate (huge threshold) and partial (threshold 37 rays)
    give the same colours, classes, statuses, stop reasons and step counts."""
    hs = host_scene(grt, "kerr.toml", c4_opts(grt, max_steps=100000))
    sc = grt.Scene(hs.desc_ptr(), keepalive=hs)
    try:
        _set_tail(grt, 0)
        base, n0 = _render(grt, sc, rect)
        assert n0 == 0
        assert base.steps.max() > 50000  # the crop has long rays
        for mode in (-1, 1 << 40, 37):
            _set_tail(grt, mode)
            got, handed = _render(grt, sc, rect)
            assert handed > 0, mode
            if mode != 37:
                assert handed > 0.5 * (base.steps > 20000).sum(), (mode, handed)
            assert np.array_equal(got.xyza64, base.xyza64), mode
            assert np.array_equal(got.xyza, base.xyza), mode
            for f in ("ray_class", "status", "steps", "stop_reason"):
                assert np.array_equal(getattr(got, f), getattr(base, f)), (mode, f)
            assert got.stats["accepted_steps"] == base.stats["accepted_steps"]
            assert got.stats["attempts"] == base.stats["attempts"]
            assert got.stats["rays"] == base.stats["rays"]
    finally:
        _set_tail(grt, -1)


@pytest.mark.gpu
def test_tail_hand_off_is_bit_identical_volumetric(grt, gpu):
    """kerr-volumetric-stony.toml (Kerr-Schild + VolumetricDisc) with C4's camera: the
    handed-off rays keep their volumetric window records (chord directions, frequency
    data), so the raymarch jobs, samples and the composited frame are unchanged."""
    hs = host_scene(grt, "kerr-volumetric-stony.toml", c4_opts(grt, width=128, height=128, max_steps=100000))
    sc = grt.Scene(hs.desc_ptr(), keepalive=hs)
    rect = (0, 0, 128, 128)
    try:
        _set_tail(grt, 0)
        base, n0 = _render(grt, sc, rect)
        assert n0 == 0
        assert base.steps.max() > 50000 and base.stats["march_jobs"] > 0
        for mode in (-1, 1 << 40, 37):
            _set_tail(grt, mode)
            got, handed = _render(grt, sc, rect)
            assert handed > 0, mode
            assert np.array_equal(got.xyza64, base.xyza64), mode
            for f in ("ray_class", "status", "steps", "stop_reason"):
                assert np.array_equal(getattr(got, f), getattr(base, f)), (mode, f)
            for k in ("accepted_steps", "attempts", "rays", "march_jobs", "march_samples", "march_noise_samples",
                      "march_emit_samples"):
                assert got.stats[k] == base.stats[k], (mode, k)
    finally:
        _set_tail(grt, -1)
