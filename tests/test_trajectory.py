"""Whole-trajectory export: `render-ray` / `render-ray-at`
(main.rs:117-171), Integrator::integrate keeping every Step (integrator.rs:78-174) and
IntegratedRay::save (ray.rs:35-54).

CPU: the Rust-Display number format, the CSV writer, render_ray_at's initial momentum
(grt_ray_at: null, future-directed, the requested local direction) and the CLI's
argument errors.  GPU: the trajectory kernel against the oracle's Integrator, record
by record, bit for bit (t, native-chart position, momentum_from_state, step count,
stop reason), for camera pixels of C1-C4 and for render_ray_at rays; the reference's
own render_ray_at tests (10 steps -> header + 10 lines) through the `grt` CLI.
"""
import math
import re
import struct
import subprocess

import numpy as np
import pytest

from conftest import RESOURCES, ROOT, SCENES, c1_opts, c2_opts, c3_opts, c4_opts, host_scene

GRT = ROOT / "gr_raytracer_amd" / "lib" / "grt"


def rust_display(v: float) -> str:
    """Rust's `{}` for f64: shortest round-trip digits (Python's repr), positional."""
    v = float(v)
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "inf" if v > 0 else "-inf"
    r = repr(v)
    sign = "-" if r.startswith("-") else ""
    mant, _, exp = r.lstrip("-").partition("e")
    ip, _, fp = mant.partition(".")
    raw = ip + fp
    digits = raw.lstrip("0")
    point = len(ip) + (int(exp) if exp else 0) - (len(raw) - len(digits))  # digits before the point
    digits = digits.rstrip("0")
    if not digits:
        return sign + "0"
    n = len(digits)
    if point <= 0:
        return sign + "0." + "0" * (-point) + digits
    if point >= n:
        return sign + digits + "0" * (point - n)
    return sign + digits[:point] + "." + digits[point:]


def test_number_format_is_rust_display(grt):
    rng = np.random.default_rng(3)
    vals = [0.0, -0.0, 1.0, 0.1, 1e-7, 1e21, 1e22, 123.456, 5e-324, 1.7976931348623157e308, 2.5, -17.0,
            0.30000000000000004, float("nan"), float("inf"), -float("inf"), 1e16, 9007199254740993.0]
    vals += [struct.unpack("<d", struct.pack("<Q", int(b)))[0] for b in rng.integers(0, 2**63, 3000, dtype=np.uint64)]
    vals += list(rng.standard_normal(2000) * 10.0 ** rng.integers(-12, 12, 2000))
    for v in vals:
        assert grt.format_f64(v) == rust_display(v), v
    assert grt.format_f64(1.0) == "1" and grt.format_f64(-0.0) == "-0" and grt.format_f64(1e-7) == "0.0000001"


def _cartesian(geometry, a, x):
    t, r, th, ph = x
    if geometry == 1:
        return [t, r * math.sin(th) * math.cos(ph), r * math.sin(th) * math.sin(ph), r * math.cos(th)]
    if geometry == 3:
        return [t, (r * math.cos(ph) - a * math.sin(ph)) * math.sin(th),
                (r * math.sin(ph) + a * math.cos(ph)) * math.sin(th), r * math.cos(th)]
    return list(x)


@pytest.mark.parametrize("geometry", [0, 1, 2, 3])
def test_csv_writer(grt, tmp_path, geometry):
    rng = np.random.default_rng(geometry)
    rec = rng.standard_normal((7, 9))
    rec[:, 2] = np.abs(rec[:, 2]) + 1.0  # r > 0 for the curvilinear charts
    path = tmp_path / "ray.csv"
    grt.write_trajectory_csv(path, geometry, 0.499, rec)
    lines = path.read_text().split("\n")
    assert lines[0] == "i,t,tau,x,y,z" and lines[-1] == "" and len(lines) == 2 + len(rec)
    for i, line in enumerate(lines[1:-1]):
        f = line.split(",")
        assert f[0] == str(i) and f[1] == rust_display(rec[i, 0])
        want = _cartesian(geometry, 0.499, rec[i, 1:5])
        got = [float(x) for x in f[2:]]
        assert np.allclose(got, want, rtol=1e-14, atol=1e-300), (got, want)


@pytest.mark.parametrize("geometry,radius,a", [(0, 0.0, 0.0), (1, 1.0, 0.0), (2, 1.0, 0.5), (3, 1.0, 0.5),
                                               (4, 0.0, 0.0)])
def test_ray_at_momentum_norm(grt, oracle, geometry, radius, a):
    for position, direction in [((0.0, 4.0, -18.0), (0.0, 1.0, 0.0)), ((18.0, 0.0, 0.0), (-1.0, 0.0, 0.0)),
                                ((-10.0, 3.0, 2.5), (0.3, -0.2, 0.9))]:
        pos, mom = grt.ray_at(geometry, radius, a, position, direction)
        assert np.all(np.isfinite(mom)) and np.all(np.isfinite(pos))
        n = _inner(grt, geometry, radius, a, pos, mom, mom)
        scale = abs(mom[0]) + 1.0
        # Schwarzschild's render_ray_at does not normalise the direction
        # (cli/schwarzschild.rs:100-112): g(p, p) = 1 - |d|^2 in the local frame
        want = 1.0 - float(np.dot(direction, direction)) if geometry == 1 else 0.0
        assert abs(n - want) <= 1e-12 * scale * scale, (geometry, n, want)
        if geometry == 4:  # cli/euclidean_spherical.rs: p^t = |d|, null for any |d|
            want = 0.0
            assert abs(n) <= 1e-12 * scale * scale, (geometry, n)
        if geometry == 0:  # cli/euclidean.rs:90-91: (|d|, d) at (0, position)
            d = np.array(direction)
            assert np.array_equal(mom, [math.sqrt(d @ d), *d]) and np.array_equal(pos, [0.0, *position])


def _inner(grt, geometry, radius, a, pos, v, w):
    import pyoracle as O

    b = grt.SceneBuilder(geometry, radius, a, 1e-5).integration(10, 20.0, 0.01, 1e-5)
    d = b.build()
    return O.inner_product(d, pos, v, w)


def test_ray_at_rejects_degenerate_directions(grt):
    with pytest.raises(grt.GrtError):
        grt.ray_at(0, 0.0, 0.0, (1.0, 2.0, 3.0), (0.0, 0.0, 0.0))
    with pytest.raises(grt.GrtError):
        grt.ray_at(0, 0.0, 0.0, (1.0, 2.0, 3.0), (float("nan"), 0.0, 0.0))


def _run_cli(args, **kw):
    return subprocess.run([str(GRT), *map(str, args)], capture_output=True, text=True, timeout=300, **kw)


def test_cli_argument_errors(grt, tmp_path):
    scene = f"--config-file={SCENES / 'schwarzschild.toml'}"
    r = _run_cli([scene, f"--resource-root={RESOURCES}", "render-ray", "-r", "3"])
    assert r.returncode == 2 and "--row and --col" in r.stderr
    r = _run_cli([scene, f"--resource-root={RESOURCES}", "render-ray-at", "-p", "1,2", "-d", "1,0,0",
                  "--filename", tmp_path / "x.csv"])
    assert r.returncode == 1 and "Position must be a vector of length 3" in r.stderr
    r = _run_cli([scene, f"--resource-root={RESOURCES}", "render-ray-at", "-p", "1,2,3", "-d", "1,0",
                  "--filename", tmp_path / "x.csv"])
    assert r.returncode == 1 and "Direction must be a vector of length 3" in r.stderr
    r = _run_cli([f"--resource-root={RESOURCES}", "render-ray", "-r", "1", "-c", "2"])
    assert r.returncode == 2 and "Config file is required" in r.stderr


# ------------------------------------------------------------------ GPU ----------
def _compare(gpu_rec, gpu_n, gpu_stop, gpu_status, ref, ref_stop, ref_status, exact=True):
    assert gpu_status == ref_status
    if ref_status != 0:
        return
    assert gpu_n == len(ref), (gpu_n, len(ref))
    assert gpu_stop == ref_stop
    if exact:
        assert np.array_equal(gpu_rec, ref), np.argwhere(gpu_rec != ref)[:5]
    else:
        assert np.allclose(gpu_rec, ref, rtol=1e-9, atol=1e-12)


CASES = {
    "C1": ("euclidean.toml", c1_opts, [(128, 128), (10, 200), (255, 0)]),
    "C2": ("schwarzschild.toml", c2_opts, [(750, 750), (740, 760), (0, 0), (700, 1499), (770, 745)]),
    "C3": ("kerr-bl.toml", c3_opts, [(750, 750), (760, 700), (100, 100)]),
    "C4": ("kerr.toml", c4_opts, [(100, 100), (2048, 600), (3000, 3900)]),
    "ES": ("euclidean-spherical.toml", c1_opts, [(128, 128), (10, 200), (200, 40)]),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_trace_pixels_matches_oracle_integrator(grt, oracle, gpu, case):
    toml, mk, pixels = CASES[case]
    opts = mk(grt) if case != "C3" else mk(grt, max_steps=200000)
    hs = host_scene(grt, toml, opts)
    sc = grt.Scene(hs.desc_ptr(), keepalive=hs)
    rows = np.array([p[0] for p in pixels], float)
    cols = np.array([p[1] for p in pixels], float)
    tr = sc.trace_pixels(rows, cols, capacity=40000, device=gpu)
    pos = np.array([hs.desc.camera.position[k] for k in range(4)])
    for k, (r, c) in enumerate(pixels):
        mom = oracle.camera_ray(hs.desc, r, c)
        ref, stop, status = oracle.integrate_ray(hs.desc, pos, mom, max_out=40000)
        n = int(tr.n_steps[k])
        if n > 40000:  # long ray: compare the stored prefix
            assert len(ref) == 40000
            assert np.array_equal(tr.steps[k], ref)
            continue
        _compare(tr.ray(k), n, tr.stop_reason[k], tr.status[k], ref, stop, status)


RAY_AT = [  # the reference's render_ray_at tests (cli/*.rs) plus longer rays
    (0, 0.0, 0.0, (0.0, 4.0, -18.0), (0.0, 1.0, 0.0)),
    (1, 1.0, 0.0, (0.0, 4.0, -18.0), (0.0, 1.0, 0.0)),
    (2, 1.0, 0.5, (0.0, 4.0, -18.0), (0.0, 1.0, 0.0)),
    (3, 1.0, 0.5, (18.0, 0.0, 0.0), (1.0, 0.0, 0.0)),
    (1, 1.0, 0.0, (-12.0, 1.0, 0.5), (1.0, 0.05, 0.0)),
    (3, 1.0, 0.499, (-10.0, 0.0, -0.5), (1.0, 0.1, 0.05)),
    (4, 0.0, 0.0, (0.0, 4.0, -18.0), (0.0, 1.0, 0.0)),  # EuclideanSpherical (cli/euclidean_spherical.rs)
]


@pytest.mark.gpu
@pytest.mark.parametrize("max_steps,max_radius", [(10, 20.0), (20000, 15000.0)])
def test_trace_rays_matches_oracle_integrator(grt, oracle, gpu, max_steps, max_radius):
    for geometry, radius, a, position, direction in RAY_AT:
        b = grt.SceneBuilder(geometry, radius, a, 1e-5).integration(max_steps, max_radius, 0.01, 1e-5)
        b.camera((0.0, 18.0, 0.0, 0.8) if geometry in (0, 2) else (0.0, 18.0, 1.4, 0.0),
                 grt.stationary_velocity(geometry, radius, a, (0.0, 18.0, 0.0, 0.8) if geometry in (0, 2)
                                         else (0.0, 18.0, 1.4, 0.0)), math.pi / 4, 8, 8)
        b.celestial(grt.Checker(0.0, 10, 10, (255, 255, 255), (0, 0, 0)))
        sc = b.scene()
        pos, mom = grt.ray_at(geometry, radius, a, position, direction)
        tr = sc.trace_rays(pos[None], mom[None], device=gpu)
        ref, stop, status = oracle.integrate_ray(sc.desc, pos, mom, max_out=max_steps + 1)
        # KerrBL's initial sin/cos(theta) is glibc's sincos on the device; the oracle's
        # BL-ray initial state uses separate sin and cos calls, so allow the last ulps.
        _compare(tr.ray(0), int(tr.n_steps[0]), tr.stop_reason[0], tr.status[0], ref, stop, status,
                 exact=geometry != 3)


@pytest.mark.gpu
@pytest.mark.parametrize("k,lines_expected", [(0, None), (1, 12), (2, 12), (3, None), (6, None)])
def test_cli_render_ray_at_reference_tests(grt, oracle, gpu, tmp_path, k, lines_expected):
    """cli/{schwarzschild,kerr,kerr_bl}.rs test_render_*_ray_at: max_steps 10, max_radius
    20 -> "i,t,tau,x,y,z" + 10 records + the trailing newline = 12 split lines (KerrBL's
    test checks the header only).  Every case: as many records as the oracle's run."""
    geometry, radius, a, position, direction = RAY_AT[k]
    toml = {0: "euclidean.toml", 1: "schwarzschild.toml", 2: "kerr.toml", 3: "kerr-bl.toml",
            4: "euclidean-spherical.toml"}[geometry]
    text = (SCENES / toml).read_text()  # the tests' geometry: a = 0.5, horizon_epsilon = 1e-5
    text = re.sub(r"^a\s*=.*$", f"a = {a}", text, flags=re.M)
    text = re.sub(r"^horizon_epsilon\s*=.*$", "horizon_epsilon = 1e-5", text, flags=re.M)
    cfg = tmp_path / toml
    cfg.write_text(text)
    out = tmp_path / "ray.csv"
    r = _run_cli(["--max-steps=10", "--max-radius=20", f"--config-file={cfg}", f"--resource-root={RESOURCES}",
                  "render-ray-at", "-p", ",".join(map(str, position)), "-d", ",".join(map(str, direction)),
                  "--filename", out, f"--device={gpu}"])
    assert r.returncode == 0, r.stderr
    lines = out.read_text().split("\n")
    assert lines[0] == "i,t,tau,x,y,z"
    if lines_expected is not None:
        assert len(lines) == lines_expected
    b = grt.SceneBuilder(geometry, radius, a, 1e-5).integration(10, 20.0, 0.01, 1e-5)
    pos, mom = grt.ray_at(geometry, radius, a, position, direction)
    ref, _, _ = oracle.integrate_ray(b.build(), pos, mom, max_out=11)
    assert len(lines) == len(ref) + 2


@pytest.mark.gpu
def test_cli_render_ray_csv_is_the_oracle_trajectory(grt, oracle, gpu, tmp_path):
    """`render-ray -r R -c C` on C2: the CSV is the oracle's trajectory of that camera
    pixel, step for step (Cartesian columns via Point::to_cartesian)."""
    out = tmp_path / "ray.csv"
    r = _run_cli(["--width=1500", "--height=1500", "--camera-position=-16.0,0.0,3.5", "--theta=-3.142",
                  "--max-steps=100000", f"--config-file={SCENES / 'schwarzschild.toml'}",
                  f"--resource-root={RESOURCES}", "render-ray", "-r", "740", "-c", "760", "--filename", out,
                  f"--device={gpu}"])
    assert r.returncode == 0, r.stderr
    hs = host_scene(grt, "schwarzschild.toml", c2_opts(grt))
    pos = np.array([hs.desc.camera.position[k] for k in range(4)])
    ref, stop, status = oracle.integrate_ray(hs.desc, pos, oracle.camera_ray(hs.desc, 740, 760))
    lines = out.read_text().split("\n")
    assert lines[0] == "i,t,tau,x,y,z" and len(lines) == len(ref) + 2
    for i in (0, 1, len(ref) // 2, len(ref) - 1):
        f = lines[1 + i].split(",")
        assert f[0] == str(i) and f[1] == rust_display(ref[i, 0])
        assert np.allclose([float(x) for x in f[2:]], _cartesian(1, 0.0, ref[i, 1:5]), rtol=1e-13)
