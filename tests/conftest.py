import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def ort():
    import octreeraytracer_amd
    return octreeraytracer_amd


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    return o


@pytest.fixture(scope="session")
def renderer(ort):
    r = ort.Renderer(0)
    yield r
    r.close()


@pytest.fixture(scope="session")
def scene_c1(ort):
    s = ort.random_spheres(100, 42)
    return s, ort.build_octree(s, 4, 0)


@pytest.fixture(scope="session")
def scene_c2(ort):
    s = ort.random_spheres(10000, 42)
    return s, ort.build_octree(s, 6, 0)
