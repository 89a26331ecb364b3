import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build libdk_rx.so (gfx950) and the oracle once per session (no-op when up to date)."""
    import __graft_entry__

    __graft_entry__.build()
