"""Whole-frame parity at the BASELINE configs (marker `gpu`).

The crops of tests/test_gpu_parity.py cover a few compact windows.  Here the sample is
stratified over the *whole* frame of each config, so the shadow edge, the disc rim and
the photon ring are sampled wherever they fall:

* C2 (1500^2 schwarzschild.toml, max-steps 1e5): the full frame is rendered on the GPU
  through the rectangle path (the product's frame driver), and 20 000 pixels drawn
  one per 10 x 10 stratum-cell are traced by the oracle;
* C3 (1500^2 kerr-bl.toml): as C2, 5 000 pixels;
* C4 (4096^2 kerr.toml, Kerr-Schild, max-steps 1e6): 1 024 pixels, one per 128 x 128
  cell, and 4 096 of another draw, one per 64 x 64 cell, on both sides through the
  offsets mode at the pixel centre (dx = dy = 0.5 gives
  row + 0.0, the base ray: camera.rs:247-254, KAT in tests/test_oracle_kats.py);
* C5 (1500^2 schwarzschild.toml, stock adaptive 4 x 4): the selected pixel set of
  grt_render_section equals the oracle's collect_pixels_to_supersample applied to the
  GPU's own 1-spp f64 frame (a pure function of the buffer, raytracer.rs:386-458, with
  the frame-wide 99th-percentile floor, :118-129); the unselected pixels are the 1-spp
  frame bit for bit, and 256 random selected pixels equal the oracle's 16 jittered
  sub-rays (raytracer.rs:132-159, :320-384) and their average.

The bar is check_parity's (tests/test_gpu_parity.py), applied lazily: every pixel
where the GPU and the oracle differ in colour (1e-4 relative per channel), class,
status, stop reason or step count is re-traced by the oracle under each of its
last-ulp libm probes, and must be one that some probe moves.
"""
import numpy as np
import pytest

from conftest import c2_opts, c3_opts, c4_opts, host_scene
from test_gpu_parity import ORACLE_THREADS, PROBES, agree, gpu_scene

pytestmark = pytest.mark.gpu


def stratified(rows, cols, cell, seed):
    """One pixel per cell x cell block of the frame (ragged edge blocks included)."""
    rng = np.random.default_rng(seed)
    r0 = np.arange(0, rows, cell)
    c0 = np.arange(0, cols, cell)
    R, Cc = np.meshgrid(r0, c0, indexing="ij")
    R, Cc = R.ravel(), Cc.ravel()
    hr = np.minimum(cell, rows - R)
    hc = np.minimum(cell, cols - Cc)
    return R + (rng.random(R.size) * hr).astype(np.int64), Cc + (rng.random(Cc.size) * hc).astype(np.int64)


def oracle_pixels(oracle, desc, cols, rows_idx, cols_idx, dx=None, dy=None):
    """The oracle on an explicit pixel list (offsets mode; dx = dy = 0.5 is the base ray)."""
    n = len(rows_idx)
    pix = (np.asarray(rows_idx, np.int64) * cols + np.asarray(cols_idx, np.int64)).astype(np.uint32)
    dx = np.full(n, 0.5) if dx is None else dx
    dy = np.full(n, 0.5) if dy is None else dy
    return oracle.render_pixels(desc, 0, 0, int(desc.camera.rows), cols, threads=ORACLE_THREADS,
                                offsets=(pix, dx, dy))


def _take(d, idx):
    return {k: (v[idx] if isinstance(v, np.ndarray) else v) for k, v in d.items()}


def lazy_parity(oracle, desc, cols, rows_idx, cols_idx, got, ref, dx=None, dy=None, max_sensitive=0.02):
    """check_parity with the probes run only where GPU and oracle differ."""
    ok = agree(got["xyza64"], got["ray_class"], ref)
    same = ok & (got["status"] == ref["status"]) & (got["stop"] == ref["stop"]) & (got["steps"] == ref["steps"])
    suspect = np.where(~same)[0]
    assert suspect.size <= max_sensitive * len(same), f"{suspect.size} of {len(same)} pixels differ"
    if suspect.size:
        sub = _take(ref, suspect)
        moved = np.zeros(suspect.size, bool)
        args = (rows_idx[suspect], cols_idx[suspect], None if dx is None else dx[suspect],
                None if dy is None else dy[suspect])
        try:
            for mode in PROBES:
                oracle.lib().oracle_set_libm_perturbation(mode)
                p = oracle_pixels(oracle, desc, cols, *args)
                moved |= ~agree(p["xyza"], p["ray_class"], sub) | (p["status"] != sub["status"]) | \
                    (p["stop"] != sub["stop"]) | (p["steps"] != sub["steps"])
        finally:
            oracle.lib().oracle_set_libm_perturbation(0)
        robust_wrong = suspect[~moved]
        assert robust_wrong.size == 0, (
            f"{robust_wrong.size} robust pixels differ, e.g. (row, col) "
            f"{list(zip(rows_idx[robust_wrong[:4]], cols_idx[robust_wrong[:4]]))}: "
            f"{got['xyza64'][robust_wrong[:2]]} vs {ref['xyza'][robust_wrong[:2]]}")
    # the f32 framebuffer is the f64 colour rounded once
    if "xyza" in got:
        assert np.array_equal(got["xyza"], got["xyza64"].astype(np.float32))
    return suspect


def frame_sample_check(grt, oracle, hs, cell, seed):
    sc = gpu_scene(grt, hs)
    rows, cols = sc.rows, sc.cols
    full = sc.render_pixels(0, 0, rows, cols)
    ri, ci = stratified(rows, cols, cell, seed)
    k = ri * cols + ci
    got = {"xyza": full.xyza[k], "xyza64": full.xyza64[k], "ray_class": full.ray_class[k],
           "status": full.status[k], "stop": full.stop_reason[k], "steps": full.steps[k]}
    ref = oracle_pixels(oracle, hs.desc, cols, ri, ci)
    suspect = lazy_parity(oracle, hs.desc, cols, ri, ci, got, ref)
    return len(ri), suspect.size


def test_c2_whole_frame_sample(grt, oracle, gpu):
    """configs[1]: 20 000 pixels, one per 10 x 10 cell of the 1500^2 frame."""
    n, _ = frame_sample_check(grt, oracle, host_scene(grt, "schwarzschild.toml", c2_opts(grt)), 10, 11)
    assert n == 22500 or n >= 20000


def test_c3_whole_frame_sample(grt, oracle, gpu):
    """configs[2]: 5 625 pixels, one per 20 x 20 cell."""
    n, _ = frame_sample_check(grt, oracle, host_scene(grt, "kerr-bl.toml", c3_opts(grt)), 20, 12)
    assert n >= 5000


@pytest.mark.parametrize("cell,seed", [(128, 13), (64, 17)])
def test_c4_whole_frame_sample(grt, oracle, gpu, cell, seed):
    """configs[3]: 1 024 pixels of the 4096^2 Kerr-Schild frame, one per 128 x 128 cell,
    and 4 096 more, one per 64 x 64 cell (another draw), traced in offsets mode at the
    pixel centre on both sides."""
    hs = host_scene(grt, "kerr.toml", c4_opts(grt))
    sc = gpu_scene(grt, hs)
    cols = sc.cols
    ri, ci = stratified(sc.rows, cols, cell, seed)
    pix = (ri * cols + ci).astype(np.uint32)
    half = np.full(len(pix), 0.5)
    g = sc.render_pixels(offsets=(pix, half, half))
    got = {"xyza": g.xyza, "xyza64": g.xyza64, "ray_class": g.ray_class, "status": g.status,
           "stop": g.stop_reason, "steps": g.steps}
    ref = oracle_pixels(oracle, hs.desc, cols, ri, ci)
    lazy_parity(oracle, hs.desc, cols, ri, ci, got, ref)


def test_c5_adaptive_full_frame(grt, oracle, gpu):
    """configs[4]: 1500^2 schwarzschild.toml with the stock adaptive 4 x 4 supersampling."""
    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt))
    sc = gpu_scene(grt, hs)
    ad = hs.adaptive
    assert ad.enabled == 1 and ad.samples_per_axis == 4  # the stock TOML's section
    rows, cols = sc.rows, sc.cols
    one = sc.render_pixels(0, 0, rows, cols)
    # the selection: paint-mask mode marks exactly the selected pixels (no supersampling)
    mark = np.array([-1.0, -2.0, -3.0, -4.0])  # no rendered colour is negative
    painted, cls_m, nsel_m, _ = sc.render_section(adaptive=ad, sampling_mask_xyza=mark)
    sel_gpu = np.all(painted == mark, axis=1)
    flags, _ = oracle.select_pixels(one.xyza64, one.ray_class, cols, rows, ad)
    assert nsel_m == int(sel_gpu.sum()) == int(flags.sum()) > 1000
    assert np.array_equal(sel_gpu, flags)
    # the supersampled frame
    out, cls, nsel, st = sc.render_section(adaptive=ad)
    assert nsel == nsel_m
    assert np.array_equal(cls, one.ray_class)
    keep = ~flags
    assert np.array_equal(out[keep], one.xyza64[keep])  # unselected: the 1-spp frame, bit for bit
    # 256 random selected pixels: 16 jittered sub-rays each, averaged over the OK ones
    rng = np.random.default_rng(5)
    sel_idx = np.flatnonzero(flags)
    pick = np.sort(rng.choice(sel_idx, 256, replace=False))
    spa = int(ad.samples_per_axis)
    R, Cc, DX, DY = [], [], [], []
    for p in pick:
        r, c = divmod(int(p), cols)
        for sr in range(spa):
            for sc_ in range(spa):
                dx, dy = oracle.stratified_offset(r, c, sr, sc_, spa)
                R.append(r); Cc.append(c); DX.append(dx); DY.append(dy)
    R, Cc, DX, DY = map(np.asarray, (R, Cc, DX, DY))
    ref = oracle_pixels(oracle, hs.desc, cols, R, Cc, DX, DY)
    gsub = sc.render_pixels(offsets=((R * cols + Cc).astype(np.uint32), DX, DY))
    got = {"xyza": gsub.xyza, "xyza64": gsub.xyza64, "ray_class": gsub.ray_class, "status": gsub.status,
           "stop": gsub.stop_reason, "steps": gsub.steps}
    suspect = lazy_parity(oracle, hs.desc, cols, R, Cc, got, ref, DX, DY)
    # the average (supersample, raytracer.rs:320-384): sum of the OK sub-samples in
    # stratum order, times 1 / valid
    sub_x = ref["xyza"].reshape(256, spa * spa, 4)
    sub_ok = (ref["status"] == 0).reshape(256, spa * spa)
    bad_px = set(np.unique(suspect // (spa * spa)).tolist())
    n_checked = 0
    for j, p in enumerate(pick):
        if j in bad_px:  # a libm-sensitive sub-ray moves the average; held above
            continue
        acc = np.zeros(4)
        valid = 0
        for k in range(spa * spa):
            if sub_ok[j, k]:
                acc = acc + sub_x[j, k]
                valid += 1
        want = acc * (1.0 / valid) if valid else one.xyza64[p]
        assert np.all(np.abs(out[p] - want) <= 1e-4 * np.maximum(np.abs(want), 1e-6)), (p, out[p], want)
        n_checked += 1
    assert n_checked >= 240


def test_failed_subsamples_are_reported(grt, oracle, gpu):
    """supersample's Err arm (raytracer.rs:357-362): every failed sub-sample ray is
    reported with its pixel, stratum and error, as the oracle's sub-rays say."""
    import ctypes as C
    import math

    b = grt.SceneBuilder(1, radius=2.0, horizon_epsilon=1e-4)
    b.integration(20000, 100.0, 0.01, 1e-7)
    pos = grt.cartesian_to_spherical((0.0, -16.0, 0.0, 3.5))
    vel = grt.stationary_velocity(1, 2.0, 0.0, pos)
    b.camera(pos, vel, math.pi / 4, 48, 48, 0.0, -3.142, 0.0)
    b.celestial(grt.Checker(0.0, 20.0, 20.0, (0, 255, 0), (0, 100, 0)))
    b.add_disc(3.0, 12.0, grt.BlackBody(1.0), temperature=5000.0)  # reaches inside the ISCO: BelowRISCO
    d = b.build()
    sc = grt.Scene(C.pointer(d), keepalive=(d, b))
    ad = grt.scene.default_adaptive()
    ad.enabled, ad.samples_per_axis = 1, 4
    mark = np.array([-1.0, -2.0, -3.0, -4.0])
    painted = sc.render_section_ex(adaptive=ad, sampling_mask_xyza=mark)
    sel = np.flatnonzero(np.all(painted.xyza64 == mark, axis=1))
    r = sc.render_section_ex(adaptive=ad)
    assert r.n_supersampled == sel.size > 0
    assert np.array_equal(r.status, painted.status)  # the 1-spp statuses
    # the oracle's sub-rays of every selected pixel, in (pixel, stratum) order
    R, Cc, DX, DY, KEY = [], [], [], [], []
    for p in sel:
        row, col = divmod(int(p), 48)
        for s in range(16):
            dx, dy = oracle.stratified_offset(row, col, s // 4, s % 4, 4)
            R.append(row); Cc.append(col); DX.append(dx); DY.append(dy); KEY.append(int(p) * 16 + s)
    R, Cc, DX, DY, KEY = map(np.asarray, (R, Cc, DX, DY, KEY))
    ref = oracle_pixels(oracle, d, 48, R, Cc, DX, DY)
    want = {(int(k) // 16, int(k) % 16): int(st) for k, st in zip(KEY, ref["status"]) if st != 0}
    got = {(int(p), int(s)): int(st) for p, s, st in r.failed_subsamples}
    assert r.n_failed_subsamples == len(r.failed_subsamples)
    assert len(want) > 10  # the scene does fail sub-rays
    # sorted by (pixel, stratum)
    keys = [p * 16 + s for p, s, _ in r.failed_subsamples]
    assert keys == sorted(keys)
    diff = sorted(set(want.items()) ^ set(got.items()))
    if diff:  # only libm-sensitive sub-rays may differ
        idx = np.array([int(np.flatnonzero(KEY == p * 16 + s)[0]) for (p, s), _ in diff])
        moved = np.zeros(idx.size, bool)
        try:
            for mode in PROBES:
                oracle.lib().oracle_set_libm_perturbation(mode)
                pr = oracle_pixels(oracle, d, 48, R[idx], Cc[idx], DX[idx], DY[idx])
                moved |= pr["status"] != ref["status"][idx]
        finally:
            oracle.lib().oracle_set_libm_perturbation(0)
        assert moved.all(), diff


def test_supersample_chunks_are_bit_identical(grt, gpu):
    """The supersample pass runs its selected pixels in chunks of sub-rays, each chunk's
    live count read on the device (grt_set_sub_chunk).  Forcing 7 pixels per chunk (many
    chunks, the last one partly filled, most of the worst-case chunks empty) gives the
    same frame, selection and failed sub-sample list as the default single chunk."""
    import ctypes as C
    import math

    from gr_raytracer_amd import _lib as L

    b = grt.SceneBuilder(1, radius=2.0, horizon_epsilon=1e-4)
    b.integration(20000, 100.0, 0.01, 1e-7)
    pos = grt.cartesian_to_spherical((0.0, -16.0, 0.0, 3.5))
    vel = grt.stationary_velocity(1, 2.0, 0.0, pos)
    b.camera(pos, vel, math.pi / 4, 48, 48, 0.0, -3.142, 0.0)
    b.celestial(grt.Checker(0.0, 20.0, 20.0, (0, 255, 0), (0, 100, 0)))
    b.add_disc(3.0, 12.0, grt.BlackBody(1.0), temperature=5000.0)  # BelowRISCO sub-rays
    d = b.build()
    sc = grt.Scene(C.pointer(d), keepalive=(d, b))
    ad = grt.scene.default_adaptive()
    ad.enabled, ad.samples_per_axis = 1, 4
    one = sc.render_section_ex(adaptive=ad, log_events=True)
    assert one.n_supersampled > 21 and one.n_supersampled % 7 != 0 and len(one.failed_subsamples) > 10
    try:
        L.check(L.lib().grt_set_sub_chunk(7 * 16), "grt_set_sub_chunk")
        many = sc.render_section_ex(adaptive=ad, log_events=True)
    finally:
        L.check(L.lib().grt_set_sub_chunk(0), "grt_set_sub_chunk")
    assert many.n_supersampled == one.n_supersampled
    assert np.array_equal(many.xyza64.view(np.uint64), one.xyza64.view(np.uint64))
    assert np.array_equal(many.ray_class, one.ray_class) and np.array_equal(many.status, one.status)
    assert np.array_equal(many.failed_subsamples, one.failed_subsamples)
    assert np.array_equal(many.subsample_events, one.subsample_events)
    assert many.stats["accepted_steps"] == one.stats["accepted_steps"]
