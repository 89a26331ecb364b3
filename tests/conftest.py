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
    """The library under test is the checked-out tree's build. Without a GPU (this container): build libdk_rx.so
    (gfx950) and the oracle once per session (no-op when the library's build id matches the tree). On a GPU box nothing
    is built: the session stops unless the library's id equals the tree's content hash (__graft_entry__.tree_build_id),
    and the GPU tests print the id they ran."""
    import __graft_entry__
    import torch

    if not torch.cuda.is_available():
        __graft_entry__.build()
        return
    got, want = __graft_entry__.lib_build_id(), __graft_entry__.tree_build_id()
    if got != want:
        pytest.exit(f"libdk_rx.so build id {got} != tree {want}: build on the CPU side first", returncode=3)
    print(f"\nlibdk_rx.so build id {__graft_entry__.check_loaded_build()} (= tree)")
