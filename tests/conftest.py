import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "opencv-octvr_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests through the C ABI")


@pytest.fixture(scope="session")
def product_lib():
    """Build (if needed) and load liboctvr_hip.so."""
    so = os.path.join(ROOT, "opencv-octvr_amd", "lib", "liboctvr_hip.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "opencv-octvr_amd")])
    import octvr_amd
    return octvr_amd
