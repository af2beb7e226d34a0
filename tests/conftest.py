import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("VELES_AMD_NO_SITE_CONFIG", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _pending_hip_error(request):
    """HVK_DEBUG_LAST_ERROR=1: report (and clear) a HIP error a test left
    pending on the thread - it would be charged to the next kernel-library
    launch (ops._lib reports hipGetLastError after each launch)."""
    yield
    if os.environ.get("HVK_DEBUG_LAST_ERROR") != "1" or \
            "gpu" not in request.keywords:
        return
    from veles_amd.ops import _lib
    if _lib.available():
        rc = _lib.lib().hvk_take_last_error()
        if rc:
            print("\n[pending HIP error %d after %s]" % (rc, request.node.nodeid))
