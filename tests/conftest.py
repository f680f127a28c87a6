import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "to-ued_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def pytest_collection_modifyitems(config, items):
    for item in items:
        if "gpu" in item.keywords:
            item.fixturenames.insert(0, "_require_gpu")


@pytest.fixture
def _require_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a GPU (no silent fallback: run with -m 'not gpu' on CPU)")
