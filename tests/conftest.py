import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "rust-ray-tracing_amd")
for p in (PKG, os.path.join(REPO, "tests"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def lib():
    import rt_mi355x as rt
    return rt.load_library()


@pytest.fixture(scope="session")
def renderer(lib):
    import rt_mi355x as rt
    r = rt.GpuRenderer(lib=lib)
    yield r
    r.close()
