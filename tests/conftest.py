import os
import sys

import pytest

# One HIP runtime per process: PyTorch ships its own libamdhip64.so.7 and whichever copy loads first
# serves both it and libbloomstage.so.  Loaded after the system ROCm 7.2 copy (i.e. after the first
# Stage), torch's device detection fails ("no ROCm-capable device"), so torch goes first, as it does
# in bench.py and the pipeline driver.
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libbloomstage.so on cuda:0)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session", autouse=True)
def _built_oracle():
    """The CPU checker is a prerequisite of most tests; build it if missing (gcc only)."""
    so = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    yield
