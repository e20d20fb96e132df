"""Invariant monitors (grt_health_pixels): the reference's camera-ray null check
(scene.rs:116-124) and its debug-build k.k / constants-of-motion drift monitors
(integrator.rs:91-146, report_drifts :176-201), on the GPU against the oracle's."""
import numpy as np
import pytest

from conftest import c1_opts, c2_opts, c3_opts, c4_opts, host_scene

ORACLE_THREADS = 16


def test_oracle_monitors_on_a_null_ray(grt, oracle):
    """Oracle side (CPU): camera rays are null to far below 1e-10, and along the C3 KerrBL
    rays the Carter constants stay put (the RHS integrates E, L_z, Q as constants)."""
    hs = host_scene(grt, "kerr-bl.toml", c3_opts(grt, width=64, height=64))
    per, st = oracle.health_pixels(hs.desc, 24, 24, 4, 4, threads=4)
    assert (st == 0).all()
    assert per[:, 0].max() < 1e-10
    assert np.isfinite(per).all()


@pytest.mark.gpu
@pytest.mark.parametrize("toml,opts_fn,rect", [
    ("kerr-bl.toml", c3_opts, (700, 700, 32, 32)),       # C3 crop: shadow edge + disc
    ("schwarzschild.toml", c2_opts, (700, 700, 24, 24)),  # C2
    ("kerr.toml", c4_opts, (1000, 1000, 8, 8)),           # C4 off the ring
    ("euclidean.toml", c1_opts, (100, 100, 16, 16)),      # C1
])
def test_health_counters_match_the_oracle(grt, oracle, gpu, toml, opts_fn, rect):
    hs = host_scene(grt, toml, opts_fn(grt))
    sc = grt.Scene(hs.desc_ptr(), keepalive=hs)
    h = sc.health(*rect, per_ray=True)
    ref, st = oracle.health_pixels(hs.desc, *rect, threads=ORACLE_THREADS)
    got = h["per_ray"]
    n = rect[2] * rect[3]
    assert h["rays"] == n
    assert h["failed"] == int((st != 0).sum())
    # the camera-ray null condition is pure arithmetic on the same inputs: bit-exact
    assert np.array_equal(got[:, 0], ref[:, 0])
    assert h["null_violations"] == int((ref[:, 0] >= 1e-10).sum())
    ok = st == 0
    # the drifts follow the trajectories, which match the oracle's bit for bit except on
    # libm-sensitive pixels; the maxima agree to 1e-9 relative (or 1e-18 absolute) on at
    # least 99% of the rays, and the above-1e-4 counts agree up to those rays
    close = np.all(np.abs(got - ref) <= 1e-9 * np.abs(ref) + 1e-18, axis=1)
    assert close[ok].mean() >= 0.99, close[ok].mean()
    n_far = int((~close & ok).sum())
    nc = h["n_constants"]
    assert abs(h["kk_drift_rays"] - int((ref[ok, 1] > 1e-4).sum())) <= n_far
    for c in range(nc):
        assert abs(h["constant_drift_rays"][c] - int((ref[ok, 2 + c] > 1e-4).sum())) <= n_far
    print(toml, {k: v for k, v in h.items() if k != "per_ray"})
