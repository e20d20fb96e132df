"""The Kerr-Schild work-order probe on quads (marker `gpu`): probe_quad_kernel splits each
probe ray's RHS over the 4 lanes of a quad (rhs_ks_quad, as the tail kernel does) and must
give the same keys as probe_kernel's one lane per ray, bit for bit, on the C4 layout's row
bands (kerr.toml, the C4 camera, cyclic 16-row bands; a reduced frame).  The keys only
order the tile queue, never an output; equal keys mean an unchanged queue."""
import ctypes as C

import numpy as np
import pytest

from conftest import host_scene

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("size,shard", [(512, 2), (768, 5)])
def test_probe_keys_on_quads_equal_one_lane_keys(grt, gpu, size, shard):
    import bench
    from gr_raytracer_amd import _lib as L

    opts = bench.c4_opts(grt, size)
    hs = host_scene(grt, "kerr.toml", opts)
    scene = grt.Scene(hs.desc_ptr(), keepalive=hs)
    lib = L.lib()
    sh = L.RowShard(16, shard, 8)
    rows = lib.grt_shard_row_count(size, C.byref(sh))
    n_tiles = ((rows + 7) // 8) * ((size + 7) // 8)
    fn = lib.grt_debug_probe_keys
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_int, C.POINTER(L.RowShard), C.c_int, C.c_void_p, C.c_uint64]
    keys = {}
    for quad in (0, 1):
        k = np.zeros(n_tiles, np.uint32)
        L.check(fn(scene._s, gpu, C.byref(sh), quad, k.ctypes.data, n_tiles), "grt_debug_probe_keys")
        keys[quad] = k
    assert np.array_equal(keys[0], keys[1])
    cap = int(min(32768, max(4096, 0.3 * 15000)))  # api.hip probe_cap for max_radius 15000
    assert (keys[0] > 0).all()
    assert (keys[0] >= cap).any() and (keys[0] < cap).any()  # capped probes and finished ones
    assert (keys[0] == cap - 1).any()  # probes that ended outward-bound (probe_escaped)


def _probe_keys(grt, toml, opts, shard, quad):
    from conftest import host_scene as hsc
    from gr_raytracer_amd import _lib as L

    hs = hsc(grt, toml, opts)
    scene = grt.Scene(hs.desc_ptr(), keepalive=hs)
    lib = L.lib()
    sh = L.RowShard(16, *shard)
    rows = lib.grt_shard_row_count(opts.height, C.byref(sh))
    n_tiles = ((rows + 7) // 8) * ((opts.width + 7) // 8)
    fn = lib.grt_debug_probe_keys
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_int, C.POINTER(L.RowShard), C.c_int, C.c_void_p, C.c_uint64]
    k = np.zeros(n_tiles, np.uint32)
    L.check(fn(scene._s, 0, C.byref(sh), quad, k.ctypes.data, n_tiles), "grt_debug_probe_keys")
    return k


def test_probe_keys_far_kerr_camera_keep_inward_probes(grt, gpu):
    """A Kerr-Schild camera far beyond the escape radius (r = 30 > 10 radius): a probe is
    'outward-bound' only once its r grows past where it started, so the inward probes
    run on and the horizon creepers reach the cap (keys >= cap).  With the probe's
    previous radius starting at 0, every probe ended at step 1 with the key cap - 1."""
    opts = grt.GlobalOpts(width=256, height=256, camera_position=(-30.0, 0.0, -0.5), theta=1.52, psi=-1.57,
                          phi=0.0, max_steps=1000000)
    cap = int(min(32768, max(4096, 0.3 * 15000)))
    keys = {q: _probe_keys(grt, "kerr.toml", opts, (0, 1), q) for q in (0, 1)}
    assert np.array_equal(keys[0], keys[1])
    k = keys[0]
    assert (k == cap - 1).any()  # escaping probes still end early
    assert (k >= cap).sum() >= 8  # the shadow's tiles: capped probes, keyed by their horizon distance
    assert not (k == cap - 1).all()


def test_probe_keys_schwarzschild_escaping_probes_finish_below_the_cap(grt, gpu):
    """Schwarzschild has no outward-bound shortcut, so its probe cap stays 1.3 x max_radius
    (api.hip probe_cap): an escaping probe (~max_radius unit steps) finishes below the cap
    and is keyed by its own length, under every capped probe, instead of being capped at
    0.3 x max_radius and keyed by its distance to the horizon ahead of the long rays."""
    opts = grt.GlobalOpts(width=256, height=256, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, psi=0.0, phi=0.0,
                          max_steps=1000000)
    cap = int(min(32768, max(4096, 1.3 * 15000)))
    k = _probe_keys(grt, "schwarzschild.toml", opts, (0, 1), 0)
    escaping = (k > 0.3 * 15000) & (k < cap)
    assert escaping.sum() > len(k) // 2  # most of the frame sees the celestial sphere
    assert np.median(k[escaping]) > 0.6 * 15000  # they ran out to max_radius, uncapped


@pytest.mark.gpu
def test_impact_keys_predict_escape_and_capture(grt, gpu):
    """Schwarzschild frames without the probe pass (max-steps below 8 x the probe cap) take
    their tile order from each tile's impact parameter (impact_key_kernel): the sky tiles
    of C2's camera are predicted at least max_radius steps (escaping), the tiles at the
    middle of the shadow a few hundred (captured), and the tiles at the photon ring's edge
    the longest."""
    from conftest import c2_opts

    mr = 1000.0
    opts = c2_opts(grt, width=256, height=256, max_radius=mr)
    k = _probe_keys(grt, "schwarzschild.toml", opts, (0, 1), 2).reshape(32, 32)
    assert (k[0, :] >= mr).all() and (k[:, 0] >= mr).all()  # frame border: sky
    assert k[15:17, 15:17].max() < mr  # centre of the shadow
    assert k.max() > mr + 700  # near-critical rays wind round the photon sphere


@pytest.mark.gpu
def test_impact_order_is_result_neutral(grt, gpu):
    """The impact-parameter order (automatic mode) against row-major tiles: identical frames."""
    from conftest import c2_opts
    from gr_raytracer_amd import _lib as L

    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt, width=256, height=256))
    sc = grt.Scene(hs.desc_ptr(), keepalive=hs)
    try:
        out = {}
        for mode in (-1, 0):
            L.check(L.lib().grt_set_schedule(mode))
            out[mode] = sc.render_pixels(device=gpu)
    finally:
        L.lib().grt_set_schedule(-1)
    a, b = out[-1], out[0]
    assert np.array_equal(a.xyza64, b.xyza64) and np.array_equal(a.ray_class, b.ray_class)
    assert np.array_equal(a.steps, b.steps) and np.array_equal(a.stop_reason, b.stop_reason)
    assert np.array_equal(a.status, b.status) and np.array_equal(a.hits, b.hits)
