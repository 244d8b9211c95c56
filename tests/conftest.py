import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pocket-tts_amd"))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests through the C ABI")


def load_golden(name: str) -> dict:
    from safetensors.numpy import load_file

    return load_file(str(GOLDEN / name))


@pytest.fixture(scope="session")
def oracle():
    from _oracle import Oracle

    return Oracle(0x5EED)


@pytest.fixture(scope="session")
def gpu_engine():
    """One 8-slot engine for the GPU parity tests (synthetic weights, seed 0x5EED)."""
    import pocket_tts_amd as pt

    eng = pt.Engine(device=0, max_slots=8, max_ctx=512, lsd_decode_steps=1, seed=0x5EED)
    yield eng
    eng.close()


def rms(a):
    a = np.asarray(a, np.float64)
    return float(np.sqrt(np.mean(a * a)))
