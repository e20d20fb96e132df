"""The range-free arithmetic of the render's RHS forms, on the GPU (marker `gpu`).

The Schwarzschild / KerrBL region-B RHS divide with div_inrange / div2_inrange and the
Kerr-Schild RHS with div_fx / sqrt_fx (geodesic.hip): the compiler's IEEE f64 division and
sqrt expansions without their range steps.  Their exactness argument is a case analysis of
v_div_scale / v_div_fixup over a claimed operand domain plus bound
chains from each RHS's predicate (ks_fd_ok, schw_div_ok, bl_div_ok) into that domain.  Two
checks hold them to it, bit for bit:

* test_range_free_arithmetic_map: every (exponent of x, exponent of y) cell of the whole
  f64 plane, subnormals included, with extreme and random mantissas (arith_map_kernel): no
  cell inside the claimed domain differs from the compiler's division / sqrt, and the
  measured edges of the exact region are where the case analysis puts them;
* test_rhs_fast_forms_match_ieee: the three RHS in their range-free and IEEE forms on
  >= 1M states per scene drawn at the edges of each predicate (coordinates at 0, 2^-100 and
  the cap; x^2+y^2+z^2-a^2 at its bound; r, Delta, l_z at theirs): identical outputs
  wherever the predicate admits the range-free form.
"""
import ctypes as C
import math

import numpy as np
import pytest

from conftest import c2_opts, c3_opts, c4_opts, host_scene

pytestmark = pytest.mark.gpu


def _map(grt, gpu, samples=16, seed=0x5EED):
    fn = grt._lib.lib().grt_debug_arith_map
    fn.restype = C.c_int
    fn.argtypes = [C.c_int, C.c_uint32, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
    m = np.zeros(2047 * 2047, np.uint8)
    z = np.zeros(2047, np.uint8)
    s = np.zeros(2047, np.uint8)
    assert fn(gpu, samples, seed, m.ctypes.data, z.ctypes.data, s.ctypes.data) == 0
    return m.reshape(2047, 2047), z, s


def test_range_free_arithmetic_map(grt, gpu):
    """div_inrange / div2_inrange / div_fx / sqrt_fx against the compiler's division and
    sqrt over the whole exponent plane (2047 x 2047 cells x 16 operand pairs: the four
    mantissa extremes and 12 random ones, both signs; profiles/r05a/arith_map.json).

    Exact region E of the three divisions (measured, and what the case analysis predicts):
    y normal with |y| < 2^1022 (1 / y normal), x with exponent >= -969 (biased > 53: the
    residual x - y m stays normal), exponent gap e_x - e_y within -1021 .. 1022.  In E no
    cell differs, v_div_scale's own gap trigger (>= 768) included; just outside it does:
    e_x = -970, e_y = 1022 and subnormal y.  Every bound chain of the RHS predicates lands
    in the box |x|, |y|, |x / y| within 2^+-600, far inside E."""
    m, z, s = _map(grt, gpu)
    ex, ey = np.meshgrid(np.arange(2047) - 1023, np.arange(2047) - 1023, indexing="ij")
    gap = ex - ey
    exact = (ey >= -1022) & (ey <= 1021) & (ex >= -969) & (gap >= -1021) & (gap <= 1022)
    claim = (np.abs(ex) <= 599) & (np.abs(ey) <= 599) & (np.abs(gap) <= 598)
    assert not (claim & ~exact).any()
    for bit in (1, 2, 4):
        bad = (m & bit) != 0
        assert not (bad & exact).any(), (bit, np.argwhere(exact & bad)[:5] - 1023)
        # the first failing points outside E: an exponent further and the divisions differ
        moderate = np.abs(ey) <= 500
        assert bad[(ex == -970) & moderate].any() and not bad[(ex == -969) & moderate].any()
        assert bad[(ey == 1022) & (np.abs(ex) <= 500)].any()
        assert bad[(ey == -1023) & (np.abs(ex) <= 500)].any()  # subnormal y
    # div_fx with a signed-zero numerator: exact for every normal denominator
    assert not (z[1:2046] & 8).any(), np.nonzero(z & 8)[0] - 1023
    # sqrt_fx: exact for every x >= 2^-969 (the compiler's expansion scales below 2^-767, an
    # identity down to there); the first failure is at 2^-971 (odd exponents only)
    e = np.arange(2047) - 1023
    assert not (s[e >= -969] & 16).any(), e[(s & 16) != 0]
    assert s[e == -971][0] & 16


def _check(grt, gpu, hs, states, consts=None, min_pred=0.5):
    sc = grt.Scene(hs.desc_ptr(), keepalive=hs)
    n = len(states)
    states = np.ascontiguousarray(states, np.float64)
    out = np.zeros((n, 16), np.float64)
    pred = np.zeros(n, np.uint8)
    fn = grt._lib.lib().grt_debug_rhs_check
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    cptr = None
    if consts is not None:
        consts = np.ascontiguousarray(consts, np.float64)
        cptr = consts.ctypes.data
    assert fn(sc._s, gpu, n, states.ctypes.data, cptr, out.ctypes.data, pred.ctypes.data) == 0, \
        grt._lib.lib().grt_last_error()
    fast, ieee = out[:, :8].view(np.uint64), out[:, 8:].view(np.uint64)
    both_nan = np.isnan(out[:, :8]) & np.isnan(out[:, 8:])
    same = np.all((fast == ieee) | both_nan, axis=1)
    p = pred.astype(bool)
    assert p.mean() >= min_pred, p.mean()
    bad = np.nonzero(p & ~same)[0]
    assert bad.size == 0, (bad.size, states[bad[:3]], out[bad[:3]])
    return {"states": n, "admitted": int(p.sum()), "differ_outside": int((~p & ~same).sum())}


def _edge(rng, n, lo, hi, frac_lo=0.15, frac_hi=0.15):
    """|values| log-uniform in [lo, hi), a share of them within a few ulps of either edge."""
    v = np.exp2(rng.uniform(math.log2(lo), math.log2(hi), n))
    k = rng.random(n)
    ulps = rng.integers(0, 4, n).astype(np.float64)
    v = np.where(k < frac_lo, lo * (1.0 + ulps * 2.0 ** -52), v)
    v = np.where(k > 1.0 - frac_hi, np.nextafter(hi, 0.0) * (1.0 - ulps * 2.0 ** -53), v)
    return v * rng.choice((-1.0, 1.0), n)


def _kerr_states(rng, n, a, cap):
    xyz = np.stack([_edge(rng, n, 2.0 ** -100, cap) for _ in range(3)], axis=1)
    xyz[rng.random((n, 3)) < 0.1] = 0.0
    # a quarter of the states on the x^2+y^2+z^2 - a^2 bound (ks_fd_ok: >= 2^-10 + 2^-31 rho^2)
    on = rng.random(n) < 0.25
    d = xyz[on] / np.maximum(np.linalg.norm(xyz[on], axis=1, keepdims=True), 1e-300)
    d[~np.isfinite(d).all(axis=1) | (np.linalg.norm(d, axis=1) == 0)] = (0.6, 0.0, 0.8)
    rho2 = (a * a + 2.0 ** -10) / (1.0 - 2.0 ** -31) * (1.0 + rng.integers(0, 64, on.sum()) * 2.0 ** -40)
    xyz[on] = d * np.sqrt(rho2)[:, None]
    p = rng.uniform(-4.0, 4.0, (n, 4))
    t = rng.uniform(-10.0, 10.0, (n, 1))
    return np.concatenate([t, xyz, p], axis=1)


@pytest.mark.parametrize("max_radius", [None, 3.0e9])
def test_rhs_kerr_schild_fast_form_matches_ieee(grt, gpu, max_radius):
    """rhs<KERR>'s range-free form (div_fx, sqrt_fx) against its IEEE form on 1M states at
    the edges of ks_fd_ok: each coordinate 0, near 2^-100 or just below the cap (2^15 for
    C4's max_radius 15000; 2^32, the largest cap, for max_radius 3e9), a quarter of them
    with x^2 + y^2 + z^2 - a^2 on its bound."""
    kw = {} if max_radius is None else {"max_radius": max_radius}
    hs = host_scene(grt, "kerr.toml", c4_opts(grt, width=8, height=8, **kw))
    cap = 2.0 ** (15 if max_radius is None else 32)
    if max_radius is None:
        assert hs.desc.max_radius == 15000.0  # the reference's default (cli.rs)
    a = hs.desc.a
    rng = np.random.default_rng(20251018 + (max_radius is not None))
    r = _check(grt, gpu, hs, _kerr_states(rng, 1 << 20, a, cap), min_pred=0.4)
    print("kerr-schild", max_radius, r)
    # the cap is the one the host chose: a coordinate just at it is refused
    st = _kerr_states(rng, 64, a, cap)
    st[:, 1] = cap
    sc_out = _check(grt, gpu, hs, st, min_pred=0.0)
    assert sc_out["admitted"] == 0


def test_rhs_schwarzschild_fast_form_matches_ieee(grt, gpu):
    """Region-B rhs<SCHWARZSCHILD> with div_inrange / div2_inrange against the IEEE form on
    1M states at the edges of schw_div_ok: |r| near 2^-100 and 2^100, |r - radius| near
    2^-40 radius, theta across region B (both sincos cases, and next to pi/2)."""
    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt, width=8, height=8))
    radius = hs.desc.radius
    rng = np.random.default_rng(7)
    n = 1 << 20
    r = _edge(rng, n, 2.0 ** -100, 2.0 ** 100)
    near = rng.random(n) < 0.3  # |r - radius| just above 2^-40 radius, both sides
    off = radius * 2.0 ** -40 * (1.0 + rng.integers(1, 1 << 12, near.sum()) * 2.0 ** -20)
    r[near] = radius + off * rng.choice((-1.0, 1.0), near.sum())
    theta = rng.uniform(0.86, 2.42, n)
    k = rng.random(n)
    theta = np.where(k < 0.1, math.pi / 2 + rng.integers(-8, 9, n) * 2.0 ** -52, theta)
    theta = np.where((k >= 0.1) & (k < 0.15), rng.choice((0.855469, 2.426265), n) + rng.integers(-64, 64, n) * 1e-9,
                     theta)
    st = np.stack([rng.uniform(-1, 1, n), r, theta, rng.uniform(-3, 3, n)] + [rng.uniform(-3, 3, n) for _ in range(4)],
                  axis=1)
    print("schwarzschild", _check(grt, gpu, hs, st))


def test_rhs_kerr_bl_fast_form_matches_ieee(grt, gpu):
    """Region-B rhs<KERR_BL> with div_inrange / div2_inrange against the IEEE form on 1M
    states at the edges of bl_div_ok: |r| up to 2^100 and near the horizons (small Delta),
    |l_z| near 2^-200 and 2^100, theta across region B."""
    hs = host_scene(grt, "kerr-bl.toml", c3_opts(grt, width=8, height=8))
    radius, a = hs.desc.radius, hs.desc.a
    rng = np.random.default_rng(11)
    n = 1 << 20
    r = _edge(rng, n, 2.0 ** -20, 2.0 ** 100)
    m = radius / 2.0
    disc = math.sqrt(m * m - a * a)
    hor = rng.random(n) < 0.3  # Delta small: r next to r+ or r-
    roots = rng.choice((m + disc, m - disc), hor.sum())
    r[hor] = roots * (1.0 + rng.integers(-1 << 20, 1 << 20, hor.sum()) * 2.0 ** -52)
    lz = _edge(rng, n, 2.0 ** -200, 2.0 ** 100)
    theta = rng.uniform(0.86, 2.42, n)
    theta = np.where(rng.random(n) < 0.1, math.pi / 2 + rng.integers(-8, 9, n) * 2.0 ** -52, theta)
    st = np.stack([rng.uniform(-1, 1, n), r, theta, rng.uniform(-3, 3, n), rng.uniform(-3, 3, n),
                   rng.uniform(-3, 3, n), np.zeros(n), np.zeros(n)], axis=1)
    consts = np.stack([rng.uniform(0.1, 10.0, n), lz, rng.uniform(-10.0, 100.0, n)], axis=1)
    print("kerr-bl", _check(grt, gpu, hs, st, consts))


def _frame(grt, hs, rect, range_free):
    fn = grt._lib.lib().grt_debug_range_free
    fn.restype = C.c_int
    fn.argtypes = [C.c_int]
    assert fn(1 if range_free else 0) == 0
    try:
        sc = grt.Scene(hs.desc_ptr(), keepalive=hs)
        r = sc.render_pixels(*rect, aux=True)
    finally:
        fn(1)
    return r


@pytest.mark.parametrize("case", ["c2", "c3", "c4"])
def test_range_free_frames_equal_ieee_frames(grt, gpu, case):
    """End to end: frames rendered with the range-free divisions / square roots and with
    every one of them in the compiler's IEEE form (grt_debug_range_free(0):
    DevScene::div_fast = 0) are identical bit for bit -- colours, classes, stop reasons,
    step counts, hit counts.  C2 and C3 whole frames (configs[1], [2]); a 256^2 C4 crop
    through the shadow edge and the disc at max-steps 1e5 (configs[3]'s scene)."""
    if case == "c2":
        hs, rect = host_scene(grt, "schwarzschild.toml", c2_opts(grt)), (0, 0, 1500, 1500)
    elif case == "c3":
        hs, rect = host_scene(grt, "kerr-bl.toml", c3_opts(grt)), (0, 0, 1500, 1500)
    else:
        hs, rect = host_scene(grt, "kerr.toml", c4_opts(grt, max_steps=100000)), (1920, 1920, 256, 256)
    a = _frame(grt, hs, rect, True)
    b = _frame(grt, hs, rect, False)
    assert np.array_equal(a.xyza64.view(np.uint64), b.xyza64.view(np.uint64))
    for k in ("ray_class", "status", "stop_reason", "steps", "hits"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    print(case, "rays", a.stats["rays"], "steps", a.stats["accepted_steps"], "ms range-free / IEEE",
          round(a.stats["kernel_ms"], 1), round(b.stats["kernel_ms"], 1))
