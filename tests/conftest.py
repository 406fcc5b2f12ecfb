"""pytest configuration: markers and import paths.

`-m "not gpu"` runs on CPU (this container); `-m gpu` needs an MI355X.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ray-tracing-in-one-weekend_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); calls through the C ABI")
    config.addinivalue_line("markers", "slow: takes more than ~10 s")


@pytest.fixture(scope="session")
def rtow():
    import rtow as m
    m.lib()  # raises if librtow.so is missing
    return m


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    return oracle_lib


@pytest.fixture(scope="session")
def gpu_ctx(rtow):
    if rtow.device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu tests need an MI355X")
    ctx = rtow.Context(0)
    yield ctx
    ctx.close()
