"""The fused arithmetic mode (grt_set_arithmetic(1), csrc/device/geodesic_fused.hip).

The light charts' trace kernels built with FMA contraction: the same algorithm and
operation order, one rounding per fused multiply-add.  Its bar is the north star's, not
bit identity: every pixel where the fused frame and the oracle (the reference's algorithm
with glibc's libm) differ by more than 1e-4 relative per channel, in class or in status
must be libm-sensitive -- moved by one of the oracle's own last-ulp probes -- and the stop
reason agrees on every robust pixel.  Kerr-Schild always runs the exact kernels.
Measured price of exactness (profiles/r06c): C2 -17%, C3 -13% in
this mode.
"""
import ctypes as C

import numpy as np
import pytest

from conftest import c2_opts, c3_opts, host_scene
from test_gpu_frames import oracle_pixels, stratified
from test_gpu_parity import ORACLE_THREADS, PROBES, agree, gpu_scene  # noqa: F401


@pytest.fixture
def fused(grt):
    grt.set_arithmetic("fused")
    try:
        yield
    finally:
        grt.set_arithmetic("exact")


def test_arithmetic_mode_is_validated(grt):
    from gr_raytracer_amd import _lib as L

    lib = L.lib()
    assert lib.grt_get_arithmetic() == 0  # exact by default
    assert lib.grt_set_arithmetic(2) == -22 and lib.grt_set_arithmetic(-1) == -22
    assert lib.grt_get_arithmetic() == 0
    assert lib.grt_set_arithmetic(1) == 0 and lib.grt_get_arithmetic() == 1
    assert lib.grt_set_arithmetic(0) == 0 and lib.grt_get_arithmetic() == 0


def fused_parity(oracle, desc, cols, ri, ci, got, max_outside=0.02):
    """The north-star bar on a pixel sample: outside-the-bar pixels must be libm-sensitive."""
    ref = oracle_pixels(oracle, desc, cols, ri, ci)
    ok = agree(got["xyza64"], got["ray_class"], ref) & (got["status"] == ref["status"])
    suspect = np.where(~ok)[0]
    assert suspect.size <= max_outside * len(ok), f"{suspect.size} of {len(ok)} pixels outside 1e-4"
    robust = np.ones(len(ok), bool)
    if suspect.size:
        sub = {k: (v[suspect] if isinstance(v, np.ndarray) else v) for k, v in ref.items()}
        moved = np.zeros(suspect.size, bool)
        try:
            for mode in PROBES:
                oracle.lib().oracle_set_libm_perturbation(mode)
                p = oracle_pixels(oracle, desc, cols, ri[suspect], ci[suspect])
                moved |= ~agree(p["xyza"], p["ray_class"], sub) | (p["status"] != sub["status"])
        finally:
            oracle.lib().oracle_set_libm_perturbation(0)
        wrong = suspect[~moved]
        assert wrong.size == 0, f"{wrong.size} robust pixels outside 1e-4, e.g. {list(zip(ri[wrong[:4]], ci[wrong[:4]]))}"
        robust[suspect] = False
    assert np.array_equal(got["stop"][robust], ref["stop"][robust])
    bit_exact = np.all(got["xyza64"] == ref["xyza"], axis=1).mean()
    return ok.mean(), bit_exact


def sample_frame(sc, cell, seed):
    full = sc.render_pixels(0, 0, sc.rows, sc.cols)
    ri, ci = stratified(sc.rows, sc.cols, cell, seed)
    k = ri * sc.cols + ci
    got = {"xyza64": full.xyza64[k], "ray_class": full.ray_class[k], "status": full.status[k],
           "stop": full.stop_reason[k], "steps": full.steps[k]}
    return full, ri, ci, got


@pytest.mark.gpu
def test_fused_c1_whole_frame(grt, oracle, gpu, fused):
    hs = host_scene(grt, "euclidean.toml", grt.GlobalOpts(width=256, height=256))
    sc = gpu_scene(grt, hs)
    full, ri, ci, got = sample_frame(sc, 1, 0)
    within, bit_exact = fused_parity(oracle, hs.desc, sc.cols, ri, ci, got, max_outside=0.0)
    assert within == 1.0 and bit_exact < 0.9  # every pixel within 1e-4, most with other last bits


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["c2", "c3"])
def test_fused_whole_frame_sample(grt, oracle, gpu, fused, config):
    """C2: 22 500 pixels (one per 10 x 10 cell), C3: 5 625 (20 x 20) of the full frame."""
    toml, opts, cell = (("schwarzschild.toml", c2_opts(grt), 10) if config == "c2" else
                        ("kerr-bl.toml", c3_opts(grt), 20))
    hs = host_scene(grt, toml, opts)
    sc = gpu_scene(grt, hs)
    full, ri, ci, got = sample_frame(sc, cell, 11)
    within, bit_exact = fused_parity(oracle, hs.desc, sc.cols, ri, ci, got)
    assert within >= 0.98 and bit_exact < 0.9
    # the f32 framebuffer is still the f64 colour rounded once
    assert np.array_equal(full.xyza, full.xyza64.astype(np.float32))


@pytest.mark.gpu
def test_fused_mode_differs_from_exact_and_keeps_kerr_schild_exact(grt, gpu):
    import bench

    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt, width=256, height=256))
    sc = gpu_scene(grt, hs)
    exact = sc.render_pixels()
    grt.set_arithmetic("fused")
    try:
        fz = sc.render_pixels()
        hk = host_scene(grt, "kerr.toml", bench.c4_opts(grt, 512, max_steps=100000))
        sk = gpu_scene(grt, hk)
        k_fused = sk.render_pixels(192, 192, 96, 96)
    finally:
        grt.set_arithmetic("exact")
    k_exact = sk.render_pixels(192, 192, 96, 96)
    # the fused kernels ran: other last bits on most sky and disc pixels, the same pixels
    differ = np.any(fz.xyza64 != exact.xyza64, axis=1)
    assert differ.mean() > 0.1, differ.mean()
    assert np.array_equal(k_fused.xyza64.view(np.uint64), k_exact.xyza64.view(np.uint64))
    assert np.array_equal(k_fused.steps, k_exact.steps)


@pytest.mark.gpu
def test_fused_c5_adaptive_frame(grt, gpu):
    """C5 (stock adaptive 4 x 4): the selection reads the 1-spp frame, whose last bits
    differ; the fused frame must select nearly the same pixels and stay within 1e-4 of
    the exact frame everywhere but on a sliver of pixels (selection flips and chaotic
    grazers)."""
    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt))
    sc = gpu_scene(grt, hs)
    exact = sc.render_section_ex(adaptive=hs.adaptive)
    grt.set_arithmetic("fused")
    try:
        fz = sc.render_section_ex(adaptive=hs.adaptive)
    finally:
        grt.set_arithmetic("exact")
    from test_gpu_parity import within

    ok = within(fz.xyza64, exact.xyza64) & (fz.ray_class == exact.ray_class)
    assert abs(fz.n_supersampled - exact.n_supersampled) <= 0.01 * exact.n_supersampled
    assert (~ok).sum() <= 1e-3 * ok.size, f"{(~ok).sum()} pixels outside 1e-4"
