import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
SCENES = ROOT / "tests" / "golden" / "scenes"
RESOURCES = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def grt():
    import gr_raytracer_amd as g

    g.lib()
    return g


@pytest.fixture(scope="session")
def oracle():
    import pyoracle

    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def gpu(grt):
    if grt.device_count() < 1:
        pytest.skip("no GPU visible")
    return 0


def c2_opts(g, **kw):
    d = dict(width=1500, height=1500, camera_position=(-16.0, 0.0, 3.5), theta=-3.142, max_steps=100000)
    d.update(kw)
    return g.GlobalOpts(**d)


def c3_opts(g, **kw):
    d = dict(width=1500, height=1500, camera_position=(-10.0, 0.0, -0.5), theta=-3.14159, max_steps=1000000)
    d.update(kw)
    return g.GlobalOpts(**d)


def c4_opts(g, **kw):
    d = dict(width=4096, height=4096, camera_position=(-10.0, 0.0, -0.5), theta=1.52, psi=-1.57, max_steps=1000000)
    d.update(kw)
    return g.GlobalOpts(**d)


def c1_opts(g, **kw):
    d = dict(width=256, height=256)
    d.update(kw)
    return g.GlobalOpts(**d)


def host_scene(g, toml, opts):
    return g.HostScene(str(SCENES / toml), opts, str(RESOURCES))
