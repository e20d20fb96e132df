"""Tile queue order (grt_set_schedule, schedule.hip): the probe-ordered queue changes
which lane traces which pixel, never a result.  Every output (colour, class, status,
steps, stop reason) must be bit-identical with and without it (GPU)."""
import numpy as np
import pytest

from conftest import c2_opts, c4_opts, host_scene


@pytest.mark.gpu
@pytest.mark.parametrize("toml,mk,rect,max_steps", [
    ("kerr.toml", c4_opts, (1900, 1700, 160, 256), 300000),
    ("schwarzschild.toml", c2_opts, (600, 600, 200, 264), 100000),
])
def test_probe_order_is_result_neutral(grt, gpu, toml, mk, rect, max_steps):
    from gr_raytracer_amd import _lib as L

    hs = host_scene(grt, toml, mk(grt, max_steps=max_steps))
    sc = grt.Scene(hs.desc_ptr(), keepalive=hs)
    out = {}
    try:  # row-major tiles; probe order from one end; probe order from both ends (default)
        for mode, two in ((0, 1), (1, 0), (1, 1)):
            L.check(L.lib().grt_set_schedule(mode))
            L.check(L.lib().grt_set_two_ended(two))
            out[mode, two] = sc.render_pixels(*rect, device=gpu)
    finally:
        L.lib().grt_set_schedule(-1)
        L.lib().grt_set_two_ended(1)
    a = out[0, 1]
    for b in (out[1, 0], out[1, 1]):
        assert np.array_equal(a.xyza64, b.xyza64) and np.array_equal(a.xyza, b.xyza)
        assert np.array_equal(a.ray_class, b.ray_class) and np.array_equal(a.status, b.status)
        assert np.array_equal(a.steps, b.steps) and np.array_equal(a.stop_reason, b.stop_reason)
        assert np.array_equal(a.hits, b.hits)
        assert a.stats["accepted_steps"] == b.stats["accepted_steps"] and a.stats["rays"] == b.stats["rays"]


def test_schedule_mode_is_validated(grt):
    from gr_raytracer_amd import _lib as L

    with pytest.raises(L.GrtError):
        L.check(L.lib().grt_set_schedule(7))
    with pytest.raises(L.GrtError):
        L.check(L.lib().grt_set_two_ended(2))
