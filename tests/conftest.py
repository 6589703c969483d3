import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "mh-spgemm_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: full-size BASELINE.json configurations")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def tool():
    if not gpu_available():
        pytest.skip("no GPU")
    import mhspgemm
    t = mhspgemm.Tool(0)
    yield t
    t.close()


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
