import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "storage-engine_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: large-size test (minutes on CPU)")


@pytest.fixture(scope="session")
def oracle():
    import oracle_ct
    return oracle_ct.load()


@pytest.fixture(autouse=True)
def _gpu_tests_use_the_gpu(request):
    """GPU tests keep every build on the device: host-memory builds at or below
    lsmb_host_max_keys() would otherwise take the library's host loop (the
    threshold's own tests set it explicitly)."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    import lsmbloom
    old = lsmbloom.host_max_keys()
    lsmbloom.set_host_max_keys(0)
    try:
        yield
    finally:
        lsmbloom.set_host_max_keys(old)
