import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available() and torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session", autouse=True)
def _built_libraries():
    """Build the oracle (test infrastructure) and the product library if missing."""
    from oracle import oracle
    if not os.path.exists(oracle.LIB_PATH):
        oracle.build()
    from rust_tracer_amd import abi
    if not os.path.exists(abi.LIB_PATH):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "rust_tracer_amd", "csrc"), "-s", "-j4"],
                       check=True)
    yield
