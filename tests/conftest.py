import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def built():
    """Build the product library and the oracle once per session (CPU-only compile)."""
    import subprocess

    subprocess.check_call(["make", "-s", "-C", ROOT])
    return True
