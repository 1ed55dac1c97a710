import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "civiwave-fem_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libcwf_hip.so on cuda:0)")
    config.addinivalue_line("markers", "slow: larger sizes (still minutes at most)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle (CPU checker) and the HIP library once per session."""
    import subprocess

    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = os.path.join(ROOT, "civiwave-fem_amd", "lib", "libcwf_hip.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "civiwave-fem_amd", "csrc")], check=True)
