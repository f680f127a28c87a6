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


def test_ctypes_signatures_match_header():
    """Every entry point's ctypes argument list has the header's arity and kinds (int / long / float /
    pointer), so a signature change in include/toued.h cannot silently desynchronise the binding."""
    import ctypes
    from toued import _lib
    text = re.sub(r"/\*.*?\*/", "", (ROOT / "include" / "toued.h").read_text(), flags=re.S)
    kinds = {ctypes.c_int: "int", ctypes.c_uint32: "int", ctypes.c_long: "long", ctypes.c_float: "float",
             ctypes.c_void_p: "ptr"}
    for m in re.finditer(r"\b(?:int|size_t|const char\*)\s+(toued_\w+)\s*\(([^)]*)\)\s*;", text):
        name, args = m.group(1), m.group(2).strip()
        params = [] if args in ("", "void") else [a.strip() for a in args.split(",")]
        sig = _lib._SIGS[name]
        assert len(sig) == len(params), (name, len(params), len(sig))
        for a, t in zip(params, sig):
            want = ("ptr" if "*" in a or a.startswith("hipStream_t") else "long" if a.startswith("long")
                    else "float" if a.startswith("float") else "int" if a.split()[0] in ("int", "uint32_t") else None)
            if want is not None and t in kinds:
                assert kinds[t] == want, (name, a, kinds[t])


def test_ctx_holds_reserved_cus_per_thread():
    """toued_set_reserved_cus writes the current context: a created context starts at 0, a thread that never
    made one current sees the process default, and destroying the current context reverts to the default."""
    import threading
    from toued import _lib
    L = _lib.lib()
    default = L.toued_ctx_current()
    assert default
    prev = L.toued_set_reserved_cus(7)
    try:
        ctx = L.toued_ctx_create()
        assert ctx and ctx != default
        assert L.toued_ctx_set_current(ctx) == 0
        assert L.toued_ctx_current() == ctx
        assert L.toued_set_reserved_cus(3) == 0          # fresh context
        seen = []
        t = threading.Thread(target=lambda: seen.append((L.toued_ctx_current(), L.toued_set_reserved_cus(7))))
        t.start(); t.join()
        assert seen == [(default, 7)]                   # other thread: the default, still 7
        assert L.toued_set_reserved_cus(-5) == 3         # negative clamps to 0
        assert L.toued_set_reserved_cus(0) == 0
        assert L.toued_ctx_destroy(ctx) == 0
        assert L.toued_ctx_current() == default
        assert L.toued_ctx_set_current(None) == 0 and L.toued_ctx_destroy(None) == 0
    finally:
        assert L.toued_set_reserved_cus(prev) == 7
