"""Rays with more window intersections than the workspace keeps in slots (GRT_MAX_HITS).

The reference keeps every window's intersection in a Vec and blends all of them back to
front (scene.rs:139-152, :206-210); an error in any window voids the pixel (scene.rs:146).
The device keeps a ray's first GRT_MAX_HITS candidates in workspace slots and appends the
rest to the hit pool (HitPool, dev_scene.h), which the shade kernel walks in window order.

The scene: Kerr (Boyer-Lindquist chart, a = 0.499) with four small spheres on a ring just
outside the horizon.  A BL ray falling into the hole winds around it without bound in phi
(dphi/dr ~ a / Delta): with horizon_epsilon = 1e-6 the rays that fall in near the spheres
cross them up to ~100 times before the horizon stop.  (A Schwarzschild ray can only wind
about ln(1e16) / 2pi ~ 6 times around the photon sphere in f64, so no Schwarzschild camera
pixel gets past 16 windows with a hit.)  The variant with a Kerr-LUT disc down to r = 0.54
adds BelowRISCO / NoCircularOrbitPossible errors, some of them in windows after the 16th
hit.
"""
import ctypes as C
import math

import numpy as np
import pytest

N = 96


def winding_scene(grt, disc=False, n=N):
    b = grt.SceneBuilder(grt._lib.GEOM_KERR_BL, radius=1.0, a=0.499, horizon_epsilon=1e-6)
    b.integration(200000, 100.0, 0.01, 1e-7)
    pos = grt.cartesian_to_boyer_lindquist(0.499, (0.0, -8.0, 0.0, 0.1))
    vel = grt.stationary_velocity(grt._lib.GEOM_KERR_BL, 1.0, 0.499, pos)
    b.camera(pos, vel, math.pi / 4, n, n, 0.0, -3.142, 0.0)
    b.celestial(grt.Checker(0.0, 20.0, 20.0, (0, 255, 0), (0, 100, 0)))
    for k in range(4):
        ang = k * math.pi / 2 + 0.3
        b.add_sphere(0.2, (0.73 * math.cos(ang), 0.73 * math.sin(ang), 0.0),
                     grt.Checker(0.0, 8.0, 8.0, (255, 0, 0), (0, 0, 255)), temperature=3000.0)
    if disc:
        b.add_disc(0.54, 3.0, grt.Checker(0.0, 10.0, 10.0, (255, 255, 0), (80, 80, 0)), temperature=4000.0)
    return b.build()


def test_oracle_scene_has_rays_past_the_slots(grt, oracle):
    """CPU: the oracle (Vec of every intersection) finds hundreds of pixels with more than
    GRT_MAX_HITS windows with a hit, and late-window errors in the disc variant."""
    ref = oracle.render_pixels(winding_scene(grt), 0, 0, N, N, threads=8)
    assert (ref["hits"] > grt._lib.GRT_MAX_HITS).sum() > 300 and ref["hits"].max() > 80
    ref = oracle.render_pixels(winding_scene(grt, disc=True), 0, 0, N, N, threads=8)
    late = (ref["status"] != 0) & (ref["hits"] > grt._lib.GRT_MAX_HITS)
    assert late.sum() >= 3, late.sum()
    assert set(np.unique(ref["status"])) == {0, 2, 3}


def _render_and_check(grt, oracle, d):
    from test_gpu_parity import _desc_ptr, check_parity, oracle_pair

    sc = grt.Scene(_desc_ptr(d), keepalive=d)
    got = sc.render_pixels(0, 0, N, N)
    ref, probes = oracle_pair(oracle, d, 0, 0, N, N)
    robust = check_parity(got, ref, probes)
    assert np.array_equal(got.hits[robust], ref["hits"][robust])
    assert got.stats["hit_overflows"] == 0
    assert not np.any(got.status & grt._lib.FLAG_HIT_OVERFLOW)
    return sc, got, ref, robust


@pytest.mark.gpu
def test_windings_past_the_workspace_slots(grt, oracle, gpu):
    """Every window's hit reaches the pixel: colour, class, status, stop, steps and the
    number of windows with a hit equal the oracle's, with rays of up to ~100 hits."""
    _, got, ref, robust = _render_and_check(grt, oracle, winding_scene(grt))
    heavy = robust & (ref["hits"] > grt._lib.GRT_MAX_HITS)
    assert heavy.sum() > 300 and got.hits.max() > 80


@pytest.mark.gpu
def test_late_window_errors(grt, oracle, gpu):
    """BelowRISCO / NoCircularOrbitPossible raised in a window after the 16th hit voids the
    pixel as in the reference (the error sits in a pool record)."""
    _, got, ref, robust = _render_and_check(grt, oracle, winding_scene(grt, disc=True))
    late = robust & (ref["status"] != 0) & (ref["hits"] > grt._lib.GRT_MAX_HITS)
    assert late.sum() >= 3
    assert np.array_equal(got.status[late], ref["status"][late])


@pytest.mark.gpu
def test_full_pool(grt, gpu):
    """A pool too small for the trace: the synchronous call traces again only the pixels
    that lost candidates, growing the pool to their need (bit-identical to a roomy pool,
    and the extra rays are a subset of the heavy pixels); an async call flags exactly the
    pixels whose candidates it lost, and after grt_hit_pool_reserve the same call is
    complete."""
    import torch

    from test_gpu_parity import _desc_ptr

    L = grt._lib
    d = winding_scene(grt)
    roomy = grt.Scene(_desc_ptr(d), keepalive=d).render_pixels(0, 0, N, N)
    rect = (32, 40, 24, 24)  # the heavy band: ~250 pixels of 17..100 hits
    sel = (np.arange(N * N) // N >= rect[0]) & (np.arange(N * N) // N < rect[0] + rect[2]) & \
          (np.arange(N * N) % N >= rect[1]) & (np.arange(N * N) % N < rect[1] + rect[3])
    want_xyza, want_status = roomy.xyza[sel], roomy.status[sel]
    L.check(L.lib().grt_set_hit_pool_min(64))
    try:
        sc = grt.Scene(_desc_ptr(d), keepalive=d)  # a fresh device copy: a 64-record pool
        sync = sc.render_pixels(*rect, aux=True)
        assert np.array_equal(sync.xyza, want_xyza) and np.array_equal(sync.status, want_status)
        assert np.array_equal(sync.xyza64, roomy.xyza64[sel]) and np.array_equal(sync.hits, roomy.hits[sel])
        assert np.array_equal(sync.steps, roomy.steps[sel]) and np.array_equal(sync.stop_reason, roomy.stop_reason[sel])
        assert sync.stats["hit_overflows"] == 0
        n_rect = rect[2] * rect[3]
        heavy = roomy.hits[sel] > L.GRT_MAX_HITS
        # the first trace plus re-traces of flagged (hence heavy) pixels only, each at most
        # three times (fits / grows the pool to the subset's need / fits)
        assert n_rect < sync.stats["rays"] <= n_rect + 3 * heavy.sum(), (sync.stats["rays"], heavy.sum())

        # a row-band shard (band 8, shard 1 of 3) and an offsets list re-trace their flagged
        # pixels too: frame rows of the shard's local rows, the same (pixel, dx, dy) items
        shard = grt.Scene(_desc_ptr(d), keepalive=d).render_shard(8, 1, 3, aux=True)
        lr = np.arange(shard.steps.size // N)
        fr = ((lr // 8) * 3 + 1) * 8 + lr % 8
        rows_sel = (np.arange(N * N) // N)
        pick = np.concatenate([np.flatnonzero(rows_sel == r) for r in fr])
        assert np.array_equal(shard.xyza64, roomy.xyza64[pick]) and np.array_equal(shard.status, roomy.status[pick])
        assert shard.stats["hit_overflows"] == 0 and shard.stats["rays"] > shard.steps.size
        rng = np.random.default_rng(7)
        pix = np.flatnonzero(sel).astype(np.uint32)
        offs = (pix, rng.random(pix.size), rng.random(pix.size))
        L.check(L.lib().grt_set_hit_pool_min(1 << 20))
        want_off = grt.Scene(_desc_ptr(d), keepalive=d).render_pixels(0, 0, N, N, offsets=offs)
        L.check(L.lib().grt_set_hit_pool_min(64))
        got_off = grt.Scene(_desc_ptr(d), keepalive=d).render_pixels(0, 0, N, N, offsets=offs)
        assert np.array_equal(got_off.xyza64, want_off.xyza64) and np.array_equal(got_off.status, want_off.status)
        assert got_off.stats["rays"] > pix.size and want_off.stats["rays"] == pix.size

        sc2 = grt.Scene(_desc_ptr(d), keepalive=d)
        n = rect[2] * rect[3]
        dev = torch.device("cuda:0")
        xyza = torch.zeros((n, 4), dtype=torch.float32, device=dev)
        cls, status = (torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(2))
        stats = torch.zeros(4, dtype=torch.int64, device=dev)

        def run():
            stats.zero_()
            L.check(L.lib().grt_render_pixels_async(sc2._s, 0, None, *rect, xyza.data_ptr(), cls.data_ptr(),
                                                    status.data_ptr(), None, None, None, stats.data_ptr()),
                    "grt_render_pixels_async")
            torch.cuda.synchronize()
            return xyza.cpu().numpy(), status.cpu().numpy(), int(stats[3])

        x1, s1, lost = run()
        flagged = (s1 & L.FLAG_HIT_OVERFLOW) != 0
        assert lost == flagged.sum() > 0
        assert not np.any(flagged & ~heavy)
        assert np.array_equal(x1[~flagged], want_xyza[~flagged])
        cap = C.c_uint64()
        L.check(L.lib().grt_hit_pool_reserve(sc2._s, 0, 0, C.byref(cap)), "grt_hit_pool_reserve")
        assert cap.value > 64
        x2, s2, lost2 = run()
        assert lost2 == 0 and np.array_equal(x2, want_xyza) and np.array_equal(s2, want_status)
    finally:
        L.check(L.lib().grt_set_hit_pool_min(1 << 20))


@pytest.mark.gpu
def test_volumetric_windings(grt, oracle, gpu):
    """A VolumetricDisc in the winding region: raymarch jobs of window-nearest volumetric
    hits past the slots are pool jobs (JOB_POOL), their colours read back from the pool."""
    b = grt.SceneBuilder(grt._lib.GEOM_KERR_BL, radius=1.0, a=0.499, horizon_epsilon=1e-6)
    b.integration(200000, 100.0, 0.01, 1e-7)
    pos = grt.cartesian_to_boyer_lindquist(0.499, (0.0, -8.0, 0.0, 0.1))
    b.camera(pos, grt.stationary_velocity(grt._lib.GEOM_KERR_BL, 1.0, 0.499, pos), math.pi / 4, 64, 64, 0.0, -3.142, 0.0)
    b.celestial(grt.Checker(0.0, 20.0, 20.0, (0, 255, 0), (0, 100, 0)))
    for k in range(3):
        ang = k * math.pi / 2 + 0.3
        b.add_sphere(0.2, (0.73 * math.cos(ang), 0.73 * math.sin(ang), 0.0),
                     grt.Checker(0.0, 8.0, 8.0, (255, 0, 0), (0, 0, 255)), temperature=3000.0)
    b.add_volumetric_disc(0.6, 2.0, grt.Checker(0.0, 10.0, 10.0, (255, 255, 0), (80, 80, 0)), temperature=4000.0,
                          thickness=0.05, constant_temperature=True, max_steps=2000, step_size=0.01)
    d = b.build()
    from test_gpu_parity import _desc_ptr, check_parity, oracle_pair

    got = grt.Scene(_desc_ptr(d), keepalive=d).render_pixels(0, 0, 64, 64)
    ref, probes = oracle_pair(oracle, d, 0, 0, 64, 64)
    robust = check_parity(got, ref, probes)
    assert np.array_equal(got.hits[robust], ref["hits"][robust])
    assert (ref["hits"] > grt._lib.GRT_MAX_HITS).sum() > 100 and got.stats["march_jobs"] > 0
