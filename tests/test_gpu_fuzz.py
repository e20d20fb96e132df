"""Seeded random scenes, GPU vs oracle (marker `gpu`).

Beyond the fixed configurations (C1-C5) and the reference's KAT scenes: every
geometry (Euclidean, Schwarzschild, Kerr-Schild, KerrBL, EuclideanSpherical), random
camera placement / orientation / field of view, random Disc and Sphere placements,
Checker and BlackBody textures, beaming, step budgets.  Each 12 x 12 frame is held to
the same bar as tests/test_gpu_parity.py (check_parity: 1e-4 per channel, identical
class / status / stop reason, with the oracle's own last-ulp probes as the allowance
for libm-sensitive pixels), including pixels that end in an error status (BelowRISCO,
NoCircularOrbitPossible, MaxStepsReached).
"""
import math

import numpy as np
import pytest

from test_gpu_parity import check_parity, oracle_pair

pytestmark = pytest.mark.gpu

N_SCENES = 30


def random_scene(grt, seed):
    rng = np.random.default_rng(1000 + seed)
    geometry = int(rng.integers(0, 5))
    radius = 0.0 if geometry in (0, 4) else float(rng.choice([1.0, 2.0]))
    a = float(rng.uniform(0.0, 0.49)) * radius if geometry in (2, 3) else 0.0
    b = grt.SceneBuilder(geometry, radius=radius, a=a, horizon_epsilon=1e-4)
    max_steps = int(rng.choice([3000, 20000]))
    b.integration(max_steps, float(rng.choice([200.0, 1000.0])), 0.01, float(rng.choice([1e-5, 1e-6])))
    # camera: Cartesian position at distance 8..30 (never on the polar axis), chart per geometry
    dist = rng.uniform(8.0, 30.0)
    th = rng.uniform(0.3, math.pi - 0.3)
    ph = rng.uniform(-math.pi, math.pi)
    cart = (0.0, dist * math.sin(th) * math.cos(ph), dist * math.sin(th) * math.sin(ph), dist * math.cos(th))
    if geometry in (1, 4):
        pos = tuple(grt.cartesian_to_spherical(cart))
    elif geometry == 3:
        pos = tuple(grt.cartesian_to_boyer_lindquist(a, cart))
    else:
        pos = cart
    vel = tuple(grt.stationary_velocity(geometry, radius, a, pos))
    alpha = float(rng.uniform(math.pi / 8, math.pi / 2))
    angles = tuple(float(x) for x in rng.uniform(-math.pi, math.pi, 3))
    b.camera(pos, vel, alpha, 12, 12, *angles)
    b.celestial(grt.Checker(float(rng.choice([0.0, 3.0])), 40.0, 20.0, (0, 200, 40), (10, 60, 0)))
    inner = float(rng.uniform(1.5, 6.0)) * max(radius, 1.0)
    disc_tex = grt.BlackBody(float(rng.choice([0.0, 2.0]))) if rng.random() < 0.4 else \
        grt.Checker(0.0, 60.0, 8.0, (0, 0, 255), (0, 0, 90))
    b.add_disc(inner, inner + float(rng.uniform(1.0, 8.0)), disc_tex, float(rng.choice([0.0, 6000.0])))
    if rng.random() < 0.7:
        c = rng.normal(size=3)
        c = c / np.linalg.norm(c) * rng.uniform(4.0, 15.0)
        b.add_sphere(float(rng.uniform(0.5, 2.0)), tuple(c), grt.Checker(0.0, 10.0, 10.0, (255, 0, 0), (90, 0, 0)),
                     float(rng.choice([0.0, 4000.0])))
    return b


@pytest.mark.parametrize("seed", range(N_SCENES))
def test_random_scene_matches_oracle(grt, oracle, gpu, seed):
    import ctypes as C

    b = random_scene(grt, seed)
    d = b.build()
    sc = grt.Scene(C.pointer(d), keepalive=(d, b))
    got = sc.render_pixels(0, 0, 12, 12)
    ref, probes = oracle_pair(oracle, d, 0, 0, 12, 12)
    robust = check_parity(got, ref, probes, max_sensitive=0.15)
    assert np.array_equal(got.status[robust], ref["status"][robust])
