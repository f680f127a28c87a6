"""RL maths of util/metrics.py on MI355X.

``gae`` is util/metrics.py:17-38 (Generalized Advantage Estimation, "lifted from Gymnax-blines") for a whole batch of
workers in one launch of ``toued_gae``: one lane per worker, the reverse scan over T in the reference's operation
order.  The training kernels (k_eval_loss, k_a2c_update, k_a2c_chain) run the same scan fused on trajectories they
already hold on chip; this entry point is the reference's standalone function.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


def gae(value: torch.Tensor, reward: torch.Tensor, done: torch.Tensor, discount: float, gae_lambda: float):
    """util/metrics.py:17-38.  ``value`` has length T+1 and ``reward``/``done`` length T along the time axis, as in
    the reference.  Shapes: value [T+1], reward/done [T] (one worker, the reference's call), or the batched layout
    value [N, T+1, W], reward/done [N, T, W] (time-major within an agent, workers contiguous: the trajectory layout
    of toued.rollout).  Returns (advantages, targets) shaped like ``reward``."""
    single = value.dim() == 1
    if single:
        value, reward, done = value.view(1, -1, 1), reward.view(1, -1, 1), done.view(1, -1, 1)
    if value.dim() != 3 or reward.shape != done.shape or reward.dim() != 3:
        raise ValueError(f"gae: value {tuple(value.shape)}, reward {tuple(reward.shape)}, done {tuple(done.shape)}")
    N, T, W = reward.shape
    if value.shape != (N, T + 1, W):
        raise ValueError(f"gae: value {tuple(value.shape)} must be [N, T+1, W] = [{N}, {T + 1}, {W}]")
    if not (value.is_cuda and reward.is_cuda and done.is_cuda):
        raise ValueError("gae: device tensors expected (the HIP path has no CPU fallback)")
    value = value.contiguous().float()
    reward = reward.contiguous().float()
    done = done.contiguous().to(torch.uint8)
    adv = torch.empty_like(reward)
    target = torch.empty_like(reward)
    # discount * gae_lambda is a python-float product in the reference (weak-typed, rounded to f32 once)
    gl = float(np.float32(float(discount) * float(gae_lambda)))
    _lib.call("toued_gae", N, W, T, _lib.ptr(value), _lib.ptr(reward), _lib.ptr(done), float(discount), gl,
              _lib.ptr(adv), _lib.ptr(target), _lib.stream_ptr())
    if single:
        return adv.view(-1), target.view(-1)
    return adv, target
