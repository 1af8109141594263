import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP engine's C ABI)")
    config.addinivalue_line("markers", "slow: longer CPU statistics runs")


def gpu_available() -> bool:
    try:
        from artes_amd import engine

        return engine.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def require_gpu():
    from artes_amd import engine

    engine.lib()   # the native engine must load -- no fallback exists
    if engine.device_count() <= 0:
        pytest.skip("no HIP device visible")
    return engine
