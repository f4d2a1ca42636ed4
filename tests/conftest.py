import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtsg on a HIP device)")
    # A GPU run initialises torch's HIP runtime before libtsg's first context: the torch wheel
    # carries its own runtime, and once libtsg's has claimed the device torch's reports "No HIP
    # GPUs are available" (bench.py sets the torch device first for the same reason). Only
    # the RCCL transport test uses torch on the GPU.
    mark = getattr(config.option, "markexpr", "") or ""
    if "gpu" in mark and "not gpu" not in mark:
        try:
            import torch
            torch.cuda.init()
        except Exception:  # noqa: BLE001  (no GPU here: the gpu tests report it themselves)
            pass


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "known_answers.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def engine():
    from tempo_amd import Engine
    e = Engine()
    yield e
    e.close()
