"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: full-size (BASELINE config) sizes")


@pytest.fixture(scope="session")
def vectors():
    d = json.loads((GOLDEN / "vectors.json").read_text())
    return d


@pytest.fixture(scope="session")
def digests():
    return json.loads((GOLDEN / "digests.json").read_text())["configs"]


@pytest.fixture(scope="session")
def oracle():
    import oracle as o  # noqa: WPS433  (test infrastructure)
    o.lib()
    return o


def hexkey(v):
    return bytes.fromhex(v["key"])


def u64(s: str) -> int:
    return int(s, 16)


@pytest.fixture(scope="session")
def cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test run without a visible GPU")
    return torch.device("cuda:0")
