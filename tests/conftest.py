import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "raytracer-795_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def lib():
    import rtg
    return rtg.load_library()


@pytest.fixture(scope="session")
def gpu(lib):
    if lib.rtg_device_count() < 1:
        pytest.fail("GPU test on a machine without a HIP device")
    return 0
