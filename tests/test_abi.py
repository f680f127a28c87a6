"""libtoued_hip.so loads and exports every symbol declared in include/toued.h (no GPU calls)."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def declared_symbols():
    text = (ROOT / "include" / "toued.h").read_text()
    return sorted(set(re.findall(r"\b(toued_\w+)\s*\(", text)))


def test_header_symbols_exported():
    from toued import _lib
    L = _lib.lib()
    syms = declared_symbols()
    assert len(syms) >= 10
    for s in syms:
        assert hasattr(L, s), f"{s} declared in include/toued.h but not exported"
    assert set(syms) == set(_lib.exported_symbols()), set(syms) ^ set(_lib.exported_symbols())


def test_host_only_entry_points():
    from toued import _lib, modes
    L = _lib.lib()
    assert L.toued_abi_version() == 1
    assert L.toued_mode_program_bytes() == modes.PROGRAM_WORDS * 4
