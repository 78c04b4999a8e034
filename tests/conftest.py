import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "acquire-zarr_amd"), os.path.join(REPO, "tests"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "ref: needs the compiled reference (oracle/_ref)")


def gpu_available() -> bool:
    try:
        import aqz
        return aqz.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    import aqz
    if aqz.device_count() == 0:
        pytest.fail("gpu test selected but no HIP device is visible")
    return aqz
