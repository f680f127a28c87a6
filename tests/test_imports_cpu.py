"""Every module of the toued package imports on the CPU (no GPU call happens at import time), so that a syntax or
import error is caught here rather than on the GPU box."""
import importlib
import pkgutil
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))

import toued  # noqa: E402

MODULES = sorted(m.name for m in pkgutil.iter_modules(toued.__path__) if not m.name.startswith("lib"))  # not the HIP .so


@pytest.mark.parametrize("name", MODULES)
def test_module_imports(name):
    importlib.import_module(f"toued.{name}")
