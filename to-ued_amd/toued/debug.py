"""The reference's debug hooks (util/jax.py:5-17 jax_debug_wrapper, flags experiments/parse_args.py:7-12).

* ``--debug_nans`` sets ``jax_debug_nans`` there: the first NaN raises.  Here every stage of a meta-step that the
  reference's jitted program would produce a NaN in -- rollout rewards, the LPG's GRU states and outputs (the
  forward's relu(h) = max(h, 0) maps a NaN state to 0, so a NaN in the recurrence shows in the states first; XLA's max
  would propagate it), the agent parameters after
  the inner updates, the meta-gradient, eta after Adam, eval returns, regret scores, the ES fitness -- gets one
  device non-finite count (``toued_nonfinite_count``, stream-ordered, into its own slot of a small device array);
  the counts are read ONCE per meta-step (``NanChecker.raise_if_any``, one host sync) and the first stage in
  enqueue order with a non-finite value raises ``FloatingPointError`` with its name, as jax's does.
* ``--debug`` disables jit there (every op runs eagerly, errors surface at the op): here every C-ABI call is
  followed by ``hipDeviceSynchronize`` + ``hipGetLastError`` (``_lib.set_debug_sync``) and the device error word is
  read synchronously after each regret round.

Both cost nothing when off: ``check`` returns before touching the device.
"""
from __future__ import annotations

import torch

from . import _lib


class NanChecker:
    """Per-stage non-finite counts of one meta-step (``--debug_nans``)."""

    MAX_STAGES = 256

    def __init__(self, enabled: bool = False):
        self.enabled = bool(enabled)
        self._counts = None
        self._stages: list[str] = []

    def check(self, stage: str, *tensors) -> None:
        """Enqueue the non-finite count of each float tensor on the current stream (a no-op when disabled)."""
        if not self.enabled:
            return
        dev = next((t.device for t in tensors if torch.is_tensor(t)), None)
        if dev is None:
            return
        if self._counts is None or self._counts.device != dev:
            self._counts = torch.zeros(self.MAX_STAGES, dtype=torch.int32, device=dev)
            self._stages = []
        if len(self._stages) >= self.MAX_STAGES:
            raise RuntimeError("NanChecker: more than MAX_STAGES checks between two raise_if_any calls")
        slot = len(self._stages)
        self._stages.append(stage)
        out = self._counts.data_ptr() + 4 * slot
        for t in tensors:
            if not torch.is_tensor(t) or t.numel() == 0:
                continue
            if t.dtype != torch.float32:
                raise TypeError(f"NanChecker.check({stage!r}): float32 tensors only, got {t.dtype}")
            if t.dim() == 2 and not t.is_contiguous() and t.stride(1) == 1:   # a column block of a wider operand
                _lib.call("toued_nonfinite_count_2d", t.data_ptr(), t.shape[0], t.shape[1], t.stride(0), out,
                          _lib.stream_ptr())
                continue
            x = t if t.is_contiguous() else t.contiguous()
            _lib.call("toued_nonfinite_count", x.data_ptr(), x.numel(), out, _lib.stream_ptr())

    def raise_if_any(self) -> None:
        """Read the counts (one synchronisation) and raise at the first stage, in enqueue order, that saw a NaN/inf."""
        if not self.enabled or not self._stages:
            return
        counts = self._counts[:len(self._stages)].cpu().tolist()
        stages = self._stages
        self._counts.zero_()
        self._stages = []
        for name, c in zip(stages, counts):
            if c:
                raise FloatingPointError(f"--debug_nans: {c} non-finite value(s) at stage '{name}' "
                                         f"(first of {len(stages)} checked stages this meta-step)")


_CHECKER = NanChecker(False)
_DEBUG = False


def configure(debug: bool = False, debug_nans: bool = False) -> NanChecker:
    """Apply the reference's two flags process-wide (Trainer calls this with args.debug / args.debug_nans)."""
    global _CHECKER, _DEBUG
    _DEBUG = bool(debug)
    _lib.set_debug_sync(_DEBUG)
    _CHECKER = NanChecker(debug_nans)
    return _CHECKER


def nan_checker() -> NanChecker:
    return _CHECKER


def debug_sync() -> bool:
    return _DEBUG
