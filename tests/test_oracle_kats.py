"""The oracle against the reference's own known-answer tests (CPU, no GPU).

Each test cites the reference test it transcribes.  The reference cannot be built in
this image (no Rust toolchain, crates not vendored: SURVEY.md section 8c), so these
KATs are what pins the oracle; the GPU kernels are then checked against the oracle.
"""
import math

import numpy as np
import pytest

from conftest import SCENES

PI = math.pi


def approx_eq(a, b, eps=2.220446049250313e-16):  # approx::assert_abs_diff_eq! default epsilon
    return np.all(np.abs(np.asarray(a, float) - np.asarray(b, float)) <= eps)


# ------------------------------------------------------------- runge_kutta.rs ----
def test_rk45_analytic_ode(oracle):  # runge_kutta.rs:214-239
    for t_end in (25.0, 50.0):
        y, t = oracle.rk_analytic(t_end)
        sol = np.array([0.5 * 2.0 * t * t + 2.0 * t + 1.0, 2.0 * t + 2.0])
        assert t > t_end
        assert np.all(np.abs(y - sol) <= 1e-5), (y, sol)


# ------------------------------------------------------------------ camera.rs ----
def euclid_camera_scene(grt, position=(0.0, 1.0, 0.0, 0.0), alpha=PI / 2, rows=11, cols=11, angles=(0, 0, 0)):
    b = grt.SceneBuilder(0)
    b.integration(30000, 10000.0, 0.001, 1e-12)
    b.camera(position, (1.0, 0.0, 0.0, 0.0), alpha, rows, cols, *angles)
    b.celestial(grt.Checker(0.0, 100.0, 100.0, (0, 255, 0), (0, 100, 0)))
    return b.build()


def test_camera_corner_directions(grt, oracle):  # camera.rs:273-336
    d = euclid_camera_scene(grt)
    corner, corner_z = -0.6853582554517135, 0.24610591900311507
    cases = {(0, 0): (0.0, corner_z, -corner, corner), (0, 10): (0.0, corner_z, corner, corner),
             (5, 5): (0.0, -1.0, 0.0, 0.0), (10, 0): (0.0, corner_z, -corner, -corner),
             (10, 10): (0.0, corner_z, corner, -corner)}
    pos = (0.0, 1.0, 0.0, 0.0)
    for (r, c), want in cases.items():
        got = oracle.camera_direction(d, r, c)
        assert approx_eq(got, want), ((r, c), got, want)
        assert approx_eq(oracle.inner_product(d, pos, got, got), -1.0)


def test_centered_offset_is_base_ray(grt, oracle):  # camera.rs:338-363
    d = euclid_camera_scene(grt)
    base = oracle.camera_ray(d, 3, 7)
    centered = oracle.camera_ray(d, 3, 7, offset=(0.5, 0.5))
    assert approx_eq(base, centered)


def test_camera_rays_are_past_directed(grt, oracle):  # camera.rs:461-508
    pos = grt.cartesian_to_spherical((0.0, 10.0, 0.0, 0.0))
    b = grt.SceneBuilder(1, radius=0.0, horizon_epsilon=0.0)
    b.integration(100, 100.0, 0.01, 1e-5).camera(pos, (1.0, 0.0, 0.0, 0.0), PI / 2, 11, 11)
    b.celestial(grt.BlackBody(0.0))
    d = b.build()
    m = oracle.camera_ray(d, 5, 5)
    assert 1.0 * oracle.inner_product(d, pos, (1.0, 0.0, 0.0, 0.0), m) < 0.0
    b = grt.SceneBuilder(2, radius=0.0, a=0.0, horizon_epsilon=0.0)
    b.integration(100, 100.0, 0.01, 1e-5).camera((0.0, 10.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0), PI / 2, 11, 11)
    b.celestial(grt.BlackBody(0.0))
    d = b.build()
    m = oracle.camera_ray(d, 5, 5)
    assert -1.0 * oracle.inner_product(d, (0.0, 10.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0), m) < 0.0


def test_schwarzschild_camera_ray_is_null(grt, oracle):  # schwarzschild.rs:511-576
    pos = grt.cartesian_to_spherical((0.0, 5.0, 0.0, 0.0))
    radius = 2.0
    a = 1.0 - radius / pos[1]
    vel = (1.0 / a, -math.sqrt(radius / pos[1]), 0.0, 0.0)
    b = grt.SceneBuilder(1, radius=radius, horizon_epsilon=1e-4)
    b.integration(100, 100.0, 0.01, 1e-5).camera(pos, vel, PI / 2, 11, 11)
    b.celestial(grt.BlackBody(0.0))
    d = b.build()
    for i in range(1, 11):
        for (r, c) in ((6, i), (i, 6)):
            m = oracle.camera_ray(d, r, c)
            assert abs(oracle.inner_product(d, pos, m, m)) <= 1e-8


# ------------------------------------------------------------------- scene.rs ----
CELESTIAL_SPHERE_COLOR_2 = (0.3575761, 0.7151522, 0.119192, 1.0)
SPHERE_COLOR_2 = (0.4124564, 0.2126729, 0.0193339, 1.0)


def kat_scene(grt, geometry, radius, camera, sphere_r, disc_in, disc_out, epsilon=1e-12, horizon=1e-4):
    """test_scene::create_scene_with_camera (scene.rs:281-369)."""
    b = grt.SceneBuilder(geometry, radius=radius, horizon_epsilon=horizon)
    b.integration(30000, 10000.0, 0.001, epsilon)
    b.camera(*camera)
    b.celestial(grt.Checker(0.0, 100.0, 100.0, (0, 255, 0), (0, 100, 0)), 0.0)
    b.add_sphere(sphere_r, (0.0, 0.0, 0.0), grt.Checker(0.0, 10.0, 10.0, (255, 0, 0), (100, 0, 0)), 0.0)
    b.add_disc(disc_in, disc_out, grt.Checker(0.0, 200.0, 10.0, (0, 0, 255), (0, 0, 100)), 0.0)
    return b


KAT_SCENES = {
    # name: (builder args, pixel, expected colour, expected class or None)
    "hits_sphere": (lambda g: kat_scene(g, 0, 0.0, ((0.0, 10.0, 0.0, 0.0), (1.0, 0, 0, 0), PI / 2, 11, 11), 2.0, 0.2, 0.3),
                    (5, 5), SPHERE_COLOR_2, 2),  # scene.rs:416-438
    "hits_sphere_schwarzschild": (
        lambda g: kat_scene(g, 1, 1.0, ((0.0, 10.0, PI / 2, 0.0), (-1.0 / (1 - 0.1), -math.sqrt(0.1), 0.0, 0.0),
                                        PI / 2, 11, 11), 2.0, 3.0, 4.0), (5, 5), SPHERE_COLOR_2, None),  # :479-507
    "hits_sphere_schwarzschild_static": (
        lambda g: kat_scene(g, 1, 1.0, ((0.0, 10.0, PI / 2, 0.0), (-1.0 / math.sqrt(1 - 0.1), 0.0, 0.0, 0.0),
                                        PI / 2, 11, 11), 2.0, 3.0, 4.0), (5, 5), SPHERE_COLOR_2, None),  # :509-538
    "misses_sphere": (lambda g: kat_scene(g, 0, 0.0, ((0.0, 10.0, 0.0, 0.0), (1.0, 0, 0, 0), PI / 2, 11, 11), 2.0, 0.2, 0.3),
                      (0, 0), CELESTIAL_SPHERE_COLOR_2, 0),  # :540-563
    "misses_sphere_schwarzschild": (
        lambda g: kat_scene(g, 1, 2.0, ((0.0, 10.0, PI / 2, 0.0), (1.0 / (1 - 0.2), -math.sqrt(0.2), 0.0, 0.0),
                                        PI / 2, 11, 11, 0.0, PI / 2, PI / 2), 2.0, 3.0, 4.0),
        (0, 0), CELESTIAL_SPHERE_COLOR_2, None),  # :565-602
    "hits_horizon_schwarzschild": (
        lambda g: kat_scene(g, 1, 1.0, ((0.0, 10.0, PI / 2, PI), (-1.0 / math.sqrt(1 - 0.1), 0.0, 0.0, 0.0),
                                        PI / 2, 11, 11, PI / 2, 0.0, PI / 2), 0.5, 3.0, 4.0),
        (5, 5), (0.0, 0.0, 0.0, 1.0), 1),  # :604-633
    "hits_sphere_spherical": (  # EuclideanSpherical, camera on the -z axis (theta = pi)
        lambda g: kat_scene(g, 4, 0.0, (tuple(g.cartesian_to_spherical((0.0, 0.0, 0.0, -10.0))), (1.0, 0, 0, 0),
                                        PI / 2, 11, 11), 2.0, 0.2, 0.3),
        (5, 5), (0.052562486896837575, 0.0271025410675224, 0.002463867369774764, 1.0), None),  # :440-478
    "intersects_with_disk": (
        lambda g: kat_scene(g, 0, 0.0, ((0.0, 7.0, 0.0, 0.8), (1.0, 0, 0, 0), PI / 4, 101, 101), 1.0, 2.0, 7.0),
        (0, 51), (0.022994536463607135, 0.009197814585442854, 0.12110455021248553, 1.0), None),  # :635-666
}


def kat_desc(grt, name):
    build, pixel, want, cls = KAT_SCENES[name]
    b = build(grt)
    if name == "hits_horizon_schwarzschild":  # camera position = cartesian_to_spherical(0,-10,0,0)
        pos = grt.cartesian_to_spherical((0.0, -10.0, 0.0, 0.0))
        cam = b.d.camera
        b.camera(pos, (-1.0 / math.sqrt(1 - 0.1), 0.0, 0.0, 0.0), PI / 2, 11, 11, PI / 2, 0.0, PI / 2)
    if name == "misses_sphere_schwarzschild":
        pos = grt.cartesian_to_spherical((0.0, 10.0, 0.0, 0.0))
        a = 1.0 - 2.0 / pos[1]
        b.camera(pos, (1.0 / a, -math.sqrt(2.0 / pos[1]), 0.0, 0.0), PI / 2, 11, 11, 0.0, PI / 2, PI / 2)
    return b, pixel, want, cls


@pytest.mark.parametrize("name", sorted(KAT_SCENES))
def test_color_of_ray_kats(grt, oracle, name):
    b, pixel, want, cls = kat_desc(grt, name)
    d = b.build()
    r = oracle.color_of_ray(d, *pixel)
    assert r["status"] == 0
    assert np.all(np.abs(r["xyza"] - np.array(want)) <= 1e-6), (name, r)
    if cls is not None:
        assert r["ray_class"] == cls, (name, r)
    if name == "hits_horizon_schwarzschild":
        assert list(r["xyza"]) == [0.0, 0.0, 0.0, 1.0]


# -------------------------------------------------------------- schwarzschild.rs --
def binet_rk4(radius, r0, l, e, max_steps, step, celestial=10000.0):  # schwarzschild.rs:327-378, :857-872
    def f(y):
        u, du = y
        return np.array([du, -u + 3.0 * (radius / 2.0) * u ** 2])
    u0 = 1.0 / r0
    b = l / e
    y = np.array([u0, math.sqrt(1.0 / b ** 2 - u0 ** 2 * (1.0 - radius * u0))])
    t, out = 0.0, [(0.0, u0)]
    h = step
    for _ in range(1, max_steps):
        k1 = f(y)
        k2 = f(y + 0.5 * h * k1)
        k3 = f(y + 0.5 * h * k2)
        k4 = f(y + h * k3)
        y = y + h / 6.0 * (k1 + 2.0 * k2 + 2.0 * k3 + k4)
        t += h
        out.append((t, y[0]))
        if 1.0 / y[0] >= celestial:
            break
    return out


def compared_trajectories(grt, oracle, e, l, max_steps):  # schwarzschild.rs:740-793
    radius = 1.0
    r = 5.0
    a = 1.0 - radius / r
    b = grt.SceneBuilder(1, radius=radius, horizon_epsilon=1e-4)
    b.integration(30000, 10000.0, 0.001, 1e-12)
    b.camera((0.0, r, PI / 2, 0.0), (1.0 / math.sqrt(a), 0.0, 0.0, 0.0), PI / 4, 500, 500)
    b.celestial(grt.BlackBody(0.0))
    d = b.build()
    mom = (e / a, -math.sqrt(e * e - a * (l * l / (r * r))), 0.0, l / (r * r))
    traj, stop, status = oracle.integrate_ray(d, (0.0, r, PI / 2, 0.0), mom)
    binet = binet_rk4(radius, r, l, e, max_steps, 0.01)
    pts_a = [(s[2], s[4]) for s in traj]  # (r, phi)
    pts_b = [(1.0 / u, phi) for phi, u in binet]
    matches, pos_b = 0, 0
    for ra, pa in pts_a:
        for i in range(pos_b, len(pts_b)):
            rb, pb = pts_b[i]
            if abs(ra - rb) < 0.1 and abs(pa - pb) < 0.1:
                matches += 1
                pos_b = i + 1
                break
    return traj, stop, matches


def test_trajectory_matches_binet_escaping(grt, oracle):  # schwarzschild.rs:667-691
    traj, stop, matches = compared_trajectories(grt, oracle, 1.0, 5.0, 450)
    assert abs(traj[-1][2] - 10000.0) <= 100.0
    assert matches >= 200, matches
    assert stop == 2  # CelestialSphereReached


def test_trajectory_matches_binet_towards_black_hole(grt, oracle):  # schwarzschild.rs:693-708
    traj, stop, matches = compared_trajectories(grt, oracle, 1.0, 2.0, 450)
    assert matches >= 180, matches
    assert stop == 1  # HorizonReached


@pytest.mark.parametrize("grazing", [False, True])
def test_celestial_sphere_reachable_with_cli_defaults(grt, oracle, grazing):  # schwarzschild.rs:874-939
    radius, r0 = 2.0, 18.0
    b = grt.SceneBuilder(1, radius=radius, horizon_epsilon=1e-5)
    b.integration(20000, 15000.0, 0.01, 0.00001)
    a0 = 1.0 - radius / r0
    b.camera((0.0, r0, PI / 2, 0.0), (1.0 / math.sqrt(a0), 0.0, 0.0, 0.0), PI / 4, 11, 11)
    b.celestial(grt.BlackBody(0.0))
    d = b.build()
    if not grazing:
        mom = (1.0, a0, 0.0, 0.0)
    else:
        r_ph = 1.5 * radius
        b_crit = r_ph / math.sqrt(1.0 - radius / r_ph)
        l = b_crit * 1.001
        p_r_sq = 1.0 - a0 * l * l / (r0 * r0)
        mom = (1.0 / a0, -math.sqrt(max(p_r_sq, 0.0)), 0.0, l / (r0 * r0))
    traj, stop, status = oracle.integrate_ray(d, (0.0, r0, PI / 2, 0.0), mom)
    assert status == 0 and stop == 2, (stop, status, len(traj))


# ------------------------------------------------------------- circular_orbit.rs --
def test_r_isco_known_values(grt):  # circular_orbit.rs:150-157
    assert abs(grt.r_isco(1.0, 0.0) - 3.0) <= 1e-12
    assert 0.5 < grt.r_isco(1.0, 0.499) < 0.63


def test_killing_coefficients_closed_forms(oracle):  # circular_orbit.rs:159-177
    r_s, r = 1.0, 5.0
    m = 0.5 * r_s
    rc, ut, uphi = oracle.killing_coefficients(r_s, 0.0, r)
    assert rc == 0
    assert abs(ut - 1.0 / math.sqrt(1.0 - 3.0 * m / r)) <= 1e-14
    assert abs(uphi / ut - math.sqrt(m / r ** 3)) <= 1e-14
    assert oracle.killing_coefficients(1.0, 0.0, 1.4)[0] == 2  # NoCircularOrbitPossible
    assert oracle.killing_coefficients(1.0, 0.0, 1.6)[0] == 0


# ---------------------------------------------------- black_body_radiation.rs ----
def xyz_to_srgb(c, exposure):  # color.rs:204-234 (no tone mapping)
    m = [[3.2406255, -1.5372080, -0.4986286], [-0.9689307, 1.8757561, 0.0415175],
         [0.0557101, -0.2040211, 1.0569959]]
    out = []
    for i in range(3):
        s = m[i][0] * c[0]
        s = m[i][1] * c[1] + s
        s = m[i][2] * c[2] + s
        v = max(s * exposure, 0.0)
        enc = 12.92 * v if v <= 0.0031308 else 1.055 * math.pow(v, 1.0 / 2.4) - 0.055
        enc = min(max(enc, 0.0), 1.0)
        out.append(int(math.floor(enc * 255.0 + 0.5)))
    return tuple(out)


@pytest.mark.parametrize("temperature,rgb", [(1000.0, (255, 60, 0)), (10000.0, (137, 146, 172))])
def test_blackbody_srgb(grt, temperature, rgb):  # black_body_radiation.rs:63-73
    c = grt.blackbody_xyz(temperature, 1.0)
    assert xyz_to_srgb(c, 1.0 / (c[0] + c[1] + c[2])) == rgb


def test_blackbody_lut_matches_direct_integration(grt, oracle):  # texture.rs:466-487
    b = grt.SceneBuilder(0).integration(10, 10.0, 0.01, 1e-5)
    b.camera((0.0, 1.0, 0.0, 0.0), (1.0, 0, 0, 0), PI / 2, 11, 11).celestial(grt.BlackBody(0.0))
    d = b.build()
    for t in (1000.0, 5000.0, 10000.0, 100000.0):
        for z in (0.5, 1.0, 2.0):
            lut = oracle.texture_color(d, -1, 0.0, 0.0, z, t)[:3]
            direct = grt.blackbody_xyz(t, z)
            for k in range(3):
                assert abs(lut[k] - direct[k]) <= max(0.02 * max(abs(lut[k]), abs(direct[k])), 1e-14)


# -------------------------------------------------------------------- texture.rs --
def test_bitmap_bilinear_corners(grt, oracle):  # texture.rs:307-398, :489-506
    img = np.zeros((2, 2, 4), np.uint8)
    for y in range(2):
        for x in range(2):
            img[y, x] = (255, 0, 0, 128) if (x + y) % 2 == 0 else (0, 0, 255, 128)
    b = grt.SceneBuilder(0).integration(10, 10.0, 0.01, 1e-5)
    b.camera((0.0, 1.0, 0.0, 0.0), (1.0, 0, 0, 0), PI / 2, 11, 11).celestial(grt.Bitmap(3.0, img))
    d = b.build()
    red, blue = grt.srgb_to_xyza(255, 0, 0, 255), grt.srgb_to_xyza(0, 0, 255, 255)
    for (u, v), want in {(0.0, 0.0): red, (0.999, 0.999): red, (0.0, 0.999): blue, (0.999, 0.0): blue}.items():
        c = oracle.texture_color(d, -1, u, v, 1.0, 0.0)
        assert list(c[:3]) == list(want[:3]) and c[3] == 128.0 / 255.0
    c = oracle.texture_color(d, -1, 0.25, 0.25, 1.0, 0.0)
    assert list(c[:3]) == [(red[k] + blue[k]) / 2.0 for k in range(3)] and c[3] == 128.0 / 255.0


# ---------------------------------------------------------------------- color.rs --
def test_blend(oracle):  # color.rs:365-404
    bg, fg = (0.2, 0.4, 0.6, 1.0), (0.8, 0.1, 0.3, 0.0)
    assert approx_eq(oracle.blend(bg, fg), bg)
    assert approx_eq(oracle.blend((0.2, 0.4, 0.6, 0.0), fg), (0.0, 0.0, 0.0, 0.0))
    assert approx_eq(oracle.blend(bg, (0.6, 0.4, 0.2, 0.5)), (0.4, 0.4, 0.4, 1.0))


# ------------------------------------------------------------------ raytracer.rs --
def test_stratified_offsets_stay_in_their_cells(oracle):  # raytracer.rs:527-553
    n = 4
    for sr in range(n):
        for sc in range(n):
            dx, dy = oracle.stratified_offset(17, 23, sr, sc, n)
            assert sc / n <= dx < (sc + 1) / n and sr / n <= dy < (sr + 1) / n
            assert (dx, dy) == oracle.stratified_offset(17, 23, sr, sc, n)


# ---------------------------------------------------------------------- sphere.rs --
def spheres_desc(grt, centers):
    b = grt.SceneBuilder(0).integration(10, 10.0, 0.01, 1e-5)
    b.camera((0.0, 30.0, 0.0, 0.0), (1.0, 0, 0, 0), PI / 2, 11, 11).celestial(grt.BlackBody(0.0))
    for c in centers:
        b.add_sphere(1.0, c, grt.Checker(3.0, 5.0, 5.0, (100, 0, 0), (0, 100, 0)), 0.0)
    return b.build()


def test_sphere_intersections(grt, oracle):  # sphere.rs:188-246
    d = spheres_desc(grt, [(0.0, 0.0, 0.0), (5.0, 0.0, 0.0), (0.0, 0.0, 20.0)])
    assert oracle.object_intersects(d, 0, (0, 1.1, 0, 0), (0, 0.9, 0, 0))[0]
    assert not oracle.object_intersects(d, 0, (0, 1.1, 0, 0), (0, 1.01, 0, 0))[0]
    assert oracle.object_intersects(d, 1, (0, 6.1, 0, 0), (0, 5.9, 0, 0))[0]
    assert not oracle.object_intersects(d, 1, (0, 6.1, 0, 0), (0, 6.01, 0, 0))[0]
    hit, pt, t = oracle.object_intersects(d, 2, (0, 0, 0, 22.0), (0, 0, 0, 19.5))
    assert hit and abs(pt[3] - 21.0) <= 1e-9


def test_disc_intersection_with_native_spherical_steps(grt, oracle):  # objects.rs:231-276
    # a chord straddling the equatorial plane at r = 6 crosses a [4, 10] disc
    b = grt.SceneBuilder(0).integration(10, 10.0, 0.01, 1e-5)
    b.camera((0.0, 30.0, 0.0, 0.0), (1.0, 0, 0, 0), PI / 2, 11, 11).celestial(grt.BlackBody(0.0))
    b.add_disc(4.0, 10.0, grt.Checker(3.0, 5.0, 5.0, (100, 100, 100), (200, 200, 200)), 5000.0)
    d = b.build()
    s0 = grt.SceneBuilder  # noqa: F841
    a = (0.0, 6.0 * math.sin(PI / 2 - 0.3), 0.0, 6.0 * math.cos(PI / 2 - 0.3))
    e = (0.0, 6.0 * math.sin(PI / 2 + 0.3), 0.0, 6.0 * math.cos(PI / 2 + 0.3))
    hit, pt, t = oracle.object_intersects(d, 0, a, e)
    assert hit and abs(pt[3]) < 1e-12 and 0.0 <= t <= 1.0
