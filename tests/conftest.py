import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "poroelasticity-linear-solvers_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpls.so on the device)")


@pytest.fixture(scope="session")
def gpu():
    import lib._native as N
    if N.device_count() < 1:
        pytest.fail("no GPU visible to libpls.so (gpu tests must run on the MI355X box)")
    N.check(N.lib().pls_set_device(0))
    return N
