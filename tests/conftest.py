import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build librtmi.so and the oracle once per session if missing."""
    from raytracingthenextweekcuda_amd import _lib
    from oracle import oracle as orc

    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    if not os.path.exists(orc.LIB_PATH):
        orc.build()
