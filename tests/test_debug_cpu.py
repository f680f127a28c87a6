"""Host-side plumbing of the debug hooks and device errors (no GPU needed).

* util/jax.py:5-17 --debug / --debug_nans: toued.debug.configure, NanChecker's stage bookkeeping, the --debug
  per-call synchronise (_lib.call -> toued_sync_check) raising ToUEDError with toued_last_error()'s text;
* the error plumbing every ABI call shares (a refused call -> ToUEDError carrying toued_last_error());
* toued_ctx: a context current on another thread cannot be destroyed, the reserved-CU setting is
  per context.
"""
import ctypes
import threading

import numpy as np
import pytest
import torch

from toued import _lib, debug
from toued.parse_args import parse_args


@pytest.fixture(autouse=True)
def _reset_debug():
    yield
    debug.configure(False, False)


def test_flags_parsed_and_configured():
    a = parse_args(["--debug", "--debug_nans"])
    assert a.debug and a.debug_nans
    ch = debug.configure(a.debug, a.debug_nans)
    assert ch.enabled and debug.debug_sync() and debug.nan_checker() is ch
    ch = debug.configure(False, False)
    assert not ch.enabled and not debug.debug_sync()


def test_checker_off_touches_nothing(monkeypatch):
    def boom(*a):
        raise AssertionError("a disabled NanChecker must not call the library")
    monkeypatch.setattr(debug._lib, "call", boom)
    ch = debug.NanChecker(False)
    ch.check("x", torch.tensor([float("nan")]))
    ch.raise_if_any()


def _fake_count(monkeypatch):
    """Stand-in for toued_nonfinite_count on CPU tensors: reads the floats at x_ptr, adds the count at out."""
    calls = []

    def fake(name, x_ptr, n, out_ptr, stream):
        assert name == "toued_nonfinite_count"
        x = np.ctypeslib.as_array(ctypes.cast(x_ptr, ctypes.POINTER(ctypes.c_float)), shape=(n,))
        c = ctypes.cast(out_ptr, ctypes.POINTER(ctypes.c_int))
        c[0] += int((~np.isfinite(x)).sum())
        calls.append(n)
        return 0
    monkeypatch.setattr(debug._lib, "call", fake)
    monkeypatch.setattr(debug._lib, "stream_ptr", lambda: None)
    return calls


def test_checker_reports_first_stage_in_order(monkeypatch):
    calls = _fake_count(monkeypatch)
    ch = debug.NanChecker(True)
    ch.check("rollout_rewards", torch.ones(10))
    ch.check("lpg_outputs", torch.tensor([1.0, float("nan")]), torch.tensor([float("inf")]))
    ch.check("meta_gradient", torch.tensor([float("nan")] * 3))
    assert calls == [10, 2, 1, 3]
    with pytest.raises(FloatingPointError, match="2 non-finite value\\(s\\) at stage 'lpg_outputs'"):
        ch.raise_if_any()
    # the counts are cleared after a read: a clean step raises nothing
    ch.check("rollout_rewards", torch.ones(4))
    ch.raise_if_any()


def test_checker_rejects_non_float(monkeypatch):
    _fake_count(monkeypatch)
    ch = debug.NanChecker(True)
    with pytest.raises(TypeError):
        ch.check("ids", torch.ones(3, dtype=torch.int32))


def test_refused_call_raises_with_last_error():
    spec = _lib.EnvSpecC(13, 1, 2, 1)
    with pytest.raises(_lib.ToUEDError, match="toued_a2c_chain_self failed \\(-1\\): .*unsupported"):
        _lib.call("toued_a2c_chain_self", spec, None, 4, 128, 20, 339, 1, None, None, None, None, None, 0.99, 0.95,
                  0.01, 1e-3, 1e-3, 0.5, None, None, None)


def test_debug_sync_surfaces_device_errors():
    """--debug: the call itself succeeds, the synchronise after it reports the device's state (here: no device)."""
    if torch.cuda.is_available():
        pytest.skip("needs a host without a GPU (the synchronise succeeds on one)")
    assert _lib.call("toued_ctx_set_current", None) == 0   # a host-only call
    debug.configure(debug=True)
    with pytest.raises(_lib.ToUEDError, match="toued_ctx_set_current: device error after synchronize.*--debug"):
        _lib.call("toued_ctx_set_current", None)


def test_ctx_destroy_refused_while_current_elsewhere():
    L = _lib.lib()
    ctx = L.toued_ctx_create()
    assert ctx
    ready, release, done = threading.Event(), threading.Event(), threading.Event()
    seen = {}

    def other():
        L.toued_ctx_set_current(ctx)
        seen["reserve"] = L.toued_set_reserved_cus(7)
        ready.set()
        release.wait(10)
        L.toued_ctx_set_current(None)
        done.set()

    th = threading.Thread(target=other)
    th.start()
    assert ready.wait(10)
    assert L.toued_ctx_destroy(ctx) == -1
    assert b"current on 1 other thread" in L.toued_last_error()
    # this thread's default context kept its own setting
    prev = L.toued_set_reserved_cus(3)
    assert L.toued_set_reserved_cus(prev) == 3
    release.set()
    assert done.wait(10)
    th.join()
    assert seen["reserve"] == 0
    L.toued_ctx_set_current(ctx)
    assert L.toued_set_reserved_cus(0) == 7        # the value the other thread set on this context
    assert L.toued_ctx_destroy(ctx) == 0            # current only here: allowed, reverts to the default
    assert L.toued_ctx_current() != ctx
