import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import _gossip_pkg  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgossip_hip.so)")


@pytest.fixture(scope="session")
def pkg():
    return _gossip_pkg.load()


@pytest.fixture(scope="session")
def oracle():
    from oracle import lib
    lib.load()
    return lib


@pytest.fixture(scope="session")
def harness():
    from oracle import harness
    return harness
