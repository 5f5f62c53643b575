import os
import sys

import pytest

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) HIP device; calls through the C ABI")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def gpu_ctx():
    from person_capture_amd.runtime import GpuContext
    ctx = GpuContext(0)
    yield ctx
    ctx.close()
