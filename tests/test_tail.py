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


@pytest.mark.gpu
def test_c4_production_shard_matches_oracle(grt, oracle, gpu):
    """configs[3]'s production path at full max-steps (1e6): a 1/64 cyclic row-band shard
    of the 4096^2 kerr.toml frame (16-row bands, shard 0: it holds the rows through the
    hole) through grt_render_shard with everything on automatic -- the probe-ordered
    tile queue, exact-count claims and the long-ray hand-off to tail_kernel -- checked
    against the oracle on ~540 pixels stratified over the shard plus its 16 longest rays
    (the ones the hand-off carries), with check_parity's bar applied lazily
    (raytracer.rs:195-244, kerr.rs:149-241)."""
    from gr_raytracer_amd.distributed import shard_frame_rows
    from test_gpu_frames import lazy_parity, oracle_pixels, stratified

    hs = host_scene(grt, "kerr.toml", c4_opts(grt))
    sc = grt.Scene(hs.desc_ptr(), keepalive=hs)
    _set_tail(grt, -1)
    r = sc.render_shard(16, 0, 64, aux=True)
    rep = sc.tail_report(capacity=1 << 16)
    cols = sc.cols
    frame_rows = shard_frame_rows(sc.rows, 16, 0, 64)
    assert len(frame_rows) == 64 and r.steps.size == 64 * cols
    assert rep["handed_off"] > 0  # the hand-off ran
    assert r.steps.max() >= 500000  # the shard holds the long rays the hand-off exists for
    lr, ci = stratified(64, cols, 23, 17)
    k = lr * cols + ci
    longest = np.argsort(-r.steps.astype(np.int64), kind="stable")[:16]
    k = np.unique(np.concatenate([k, longest]))
    assert np.isin(longest, rep["slot"]).any()  # some of them finished in tail_kernel
    lr, ci = k // cols, k % cols
    ri = frame_rows[lr]
    got = {"xyza": r.xyza[k], "xyza64": r.xyza64[k], "ray_class": r.ray_class[k], "status": r.status[k],
           "stop": r.stop_reason[k], "steps": r.steps[k]}
    ref = oracle_pixels(oracle, hs.desc, cols, ri, ci)
    lazy_parity(oracle, hs.desc, cols, ri, ci, got, ref)
