import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU; run on the GPU box")
    config.addinivalue_line("markers", "slow: longer CPU test")


def _ensure_built():
    """Build the oracle and the product library in-tree if missing (CPU only)."""
    if not os.path.exists(os.path.join(REPO, "oracle", "build", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True, capture_output=True)
    if not os.path.exists(os.path.join(REPO, "a_dive_into_ray_tracing_amd", "lib", "librtmi.so")):
        subprocess.run(["make", "-C", os.path.join(REPO, "a_dive_into_ray_tracing_amd", "csrc"), "-j8"], check=True, capture_output=True)


_ensure_built()


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")
