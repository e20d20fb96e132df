"""The device pow (gr_raytracer_amd/csrc/device/glibc_math.h), compiled for the host,
returns glibc's pow bits on its whole fast path (CPU only).

f64::powf in the reference is glibc pow; on x86-64 with FMA glibc 2.35 runs
__pow_fma, whose operation sequence glibc_math.h restates.  The tables come from the
installed libm (tools/gen_glibc_tables.py); this test re-derives them too, so a libm
update that changes them is caught here."""
import subprocess

import pytest

from conftest import ROOT

DEV = ROOT / "gr_raytracer_amd" / "csrc" / "device"
MODES = {0: "controller eps/err over 1e-304..1e304, y = 1/5", 1: "controller range", 2: "beaming exponents",
         3: "x near 1", 4: "random normal x, |y| < 2"}


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = tmp_path_factory.mktemp("glibc") / "check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", str(DEV),
                    str(ROOT / "tests" / "native" / "glibc_pow_check.cpp"), "-o", str(exe)], check=True)
    return exe


@pytest.mark.parametrize("mode", sorted(MODES))
def test_device_pow_is_bit_identical_to_glibc(checker, mode):
    out = subprocess.run([str(checker), str(mode), "400000"], check=True, capture_output=True, text=True).stdout
    n, fast, bad = map(int, out.strip().splitlines()[-1].split())
    assert bad == 0, out
    assert fast >= 0.7 * n, (MODES[mode], fast, n)
    if mode in (0, 1):
        assert fast == n  # the controller's inputs are always on the fast path


def test_tables_match_the_installed_libm():
    gen = subprocess.run(["python3", str(ROOT / "tools" / "gen_glibc_tables.py")], check=True, capture_output=True,
                         text=True).stdout
    assert gen == (DEV / "glibc_tables.h").read_text()


TRIG_MODES = {0: "ray theta", 1: "several periods", 2: "magnitudes 2^-41..2^19", 3: "near pi/2",
              4: "up to the reduction limit", 5: "(-pi, pi): VolumetricDisc phi",
              6: "pi/2 +- 0.15 (region B, Taylor and table)"}


def _build(tmp_path_factory, name, extra=()):
    exe = tmp_path_factory.mktemp(name) / name
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", *extra, "-I", str(DEV),
                    str(ROOT / "tests" / "native" / f"{name}.cpp"), "-o", str(exe)], check=True)
    return exe


@pytest.fixture(scope="module")
def trig_checkers(tmp_path_factory):
    # -fno-builtin: sin(x) and cos(x) must reach glibc's sin / cos, not a fused sincos
    return (_build(tmp_path_factory, "glibc_trig_check", ("-fno-builtin-sin", "-fno-builtin-cos")),
            _build(tmp_path_factory, "glibc_sincos_check"))


@pytest.mark.parametrize("mode", sorted(TRIG_MODES))
def test_device_sin_cos_sincos_are_bit_identical_to_glibc(trig_checkers, mode):
    """sin_fast / cos_fast == glibc sin / cos (FMA ifunc builds); sincos_fast and its
    branch-free variant sincos_fast_uniform == glibc sincos (baseline build), on
    |x| < 105414350."""
    for exe in trig_checkers:
        out = subprocess.run([str(exe), str(mode), "300000"], check=True, capture_output=True, text=True).stdout
        n, fast, bad = map(int, out.strip().splitlines()[-1].split())
        assert bad == 0, (exe.name, out)
        assert fast == n, (exe.name, TRIG_MODES[mode], fast, n)


EXP_MODES = {0: "vertical falloff -(h/thickness)^2", 1: "boundary falloff -1/max(d^2, 1e-4)",
             2: "attenuation over 60 decades", 3: "subnormal results and the overflow edge", 4: "random bit patterns"}


@pytest.fixture(scope="module")
def exp_checker(tmp_path_factory):
    return _build(tmp_path_factory, "glibc_exp_check", ("-fno-builtin-exp",))


@pytest.mark.parametrize("mode", sorted(EXP_MODES))
def test_device_exp_is_bit_identical_to_glibc(exp_checker, mode):
    """exp_ == glibc exp (__exp_fma) on every input, including the special cases (the
    VolumetricDisc raymarch's falloffs and attenuations, volumetric_disc.rs:97-138, :242-272)."""
    out = subprocess.run([str(exp_checker), str(mode), "400000"], check=True, capture_output=True, text=True).stdout
    n, _, bad = map(int, out.strip().splitlines()[-1].split())
    assert bad == 0, (EXP_MODES[mode], out)
