import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def native():
    from dash_amd.native import native as _n

    return _n()


def pytest_collection_modifyitems(config, items):
    try:
        from dash_amd.runtime import hip_available

        has_gpu = hip_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
