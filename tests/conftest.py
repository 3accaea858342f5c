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


def record_parity_stats(name, values):
    """Statistical-tier numbers of a GPU test -> gpurun_out/parity_stats.json
    (merged back from the GPU box; copied to profiles/ per round), so the
    bias / MAE / RMSE / tile-max and convergence ratios are on record, not
    only pass/fail."""
    import json

    out = os.path.join(REPO, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, "parity_stats.json")
    data = {}
    if os.path.exists(path):
        try:
            data = json.load(open(path))
        except Exception:
            data = {}
    data[name] = {k: (round(float(v), 6) if isinstance(v, (float, int)) else v) for k, v in values.items()}
    with open(path, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")
