"""Shared fixtures. `-m gpu` tests need an MI355X (gfx950); everything else runs on CPU."""
import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests via the C ABI")


def load_golden(name):
    return json.loads((GOLDEN / name).read_text())


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def coracle():
    """The C restatement (oracle/build/liboracle.so) -- test infrastructure only."""
    from tests.oracle_c import COracle
    return COracle()


@pytest.fixture(scope="session")
def engine():
    """The product engine on cuda:0 (gpu tests only). No fallback: fails if libmde.so or the
    device is missing."""
    import mydatastore_amd as mde
    eng = mde.Engine(0)
    yield eng
    eng.close()
