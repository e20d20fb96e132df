"""Launch shape of the persistent integrate kernel (grt_set_launch_config): blocks per
CU and threads per block change which lane traces which pixel, never a result.  Every
output must be bit-identical across shapes (GPU); malformed shapes are refused (CPU)."""
import numpy as np
import pytest

from conftest import c2_opts, c4_opts, host_scene


def test_launch_config_is_validated(grt):
    lib = grt._lib.lib()
    for bpc, thr in ((-1, 256), (2, 96), (2, 512), (2, -64)):
        assert lib.grt_set_launch_config(bpc, thr) != 0, (bpc, thr)
    assert lib.grt_set_launch_config(0, 0) == 0  # back to the defaults


@pytest.mark.gpu
@pytest.mark.parametrize("toml,mk,rect", [
    ("schwarzschild.toml", c2_opts, (700, 700, 48, 64)),
    ("kerr.toml", c4_opts, (1990, 1990, 24, 24)),  # photon ring + long rays (tail hand-off)
])
def test_launch_shape_is_result_neutral(grt, gpu, toml, mk, rect):
    from gr_raytracer_amd import _lib as L

    kw = {"max_steps": 100000} if toml == "kerr.toml" else {}
    hs = host_scene(grt, toml, mk(grt, **kw))
    sc = grt.Scene(hs.desc_ptr(), keepalive=hs)
    out = {}
    try:
        for shape in ((0, 0), (1, 256), (2, 128), (8, 64), (4, 256)):
            L.check(L.lib().grt_set_launch_config(*shape))
            out[shape] = sc.render_pixels(*rect, device=gpu)
    finally:
        L.lib().grt_set_launch_config(0, 0)
    base = out[(0, 0)]
    for shape, r in out.items():
        assert np.array_equal(r.xyza64, base.xyza64), shape
        for f in ("ray_class", "status", "steps", "stop_reason"):
            assert np.array_equal(getattr(r, f), getattr(base, f)), (shape, f)
        assert r.stats["accepted_steps"] == base.stats["accepted_steps"], shape
