import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests of the HIP path")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _gpu_available() -> bool:
    try:
        from mythril_amd import _native as N

        return N.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def mgp_ctx():
    """A libmgp context on device 0 — the GPU tests fail loudly if it cannot be made."""
    from mythril_amd import _native as N

    if not _gpu_available():
        pytest.fail("gpu-marked test but no HIP device visible (libmgp has no CPU fallback)")
    ctx = N.Context(0)
    yield ctx
    ctx.close()


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
