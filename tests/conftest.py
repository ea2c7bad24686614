import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "kimera-multi_amd"))
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle
    return oracle.lib()


@pytest.fixture(scope="session")
def gpu():
    """Skip-free GPU gate: -m gpu tests must FAIL when the HIP path is missing."""
    from kmx import abi
    n = abi.device_count()
    assert n > 0, "no HIP device visible; the gpu tests need an MI355X"
    return n
