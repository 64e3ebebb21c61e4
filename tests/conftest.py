import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"
DATA_DIR = os.path.join(ROOT, "tests", "data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) HIP device")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "functional: spawns bcpd node processes")


def pytest_collection_modifyitems(config, items):
    try:
        from bitcoincashplus_amd import native
        have_gpu = bool(native.gpu_available())
    except Exception:
        have_gpu = False
    if have_gpu:
        return
    skip = pytest.mark.skip(reason="no HIP device visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def native():
    from bitcoincashplus_amd import native as n
    return n
