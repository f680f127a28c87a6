"""Agent populations on MI355X (agents/agents.py, util/data.py AgentState/Level).

An ``AgentBatch`` holds N tabular agents as dense device tensors:
  levels  int32 [N, 64]         packed Level (env params + lifetime + buffer_id)
  theta   f32   [N, D, 5]       actor Dense kernel (models/agent.py:7-17, actor_net=())
  phi     f32   [N, D, Y]       LPG target critic kernel (softmax head, critic_dims=Y)
  step    int32 [N]             TrainState.step (actor and critic step together)
  state   int32 [12, N*W]       per-worker env state (env_obs is derived: tab_idx, time)
and the value critics of the meta-gradient path: vcrit f32 [N, D], vstep int32 [N].
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib, prng
from .env import get_agent_hypers

_SQRT2 = math.sqrt(2.0)
TN_LO = float(np.float32(math.erf(-2.0 / _SQRT2)))
TN_HI = float(np.float32(math.erf(2.0 / _SQRT2)))


@dataclass
class AgentHyperparams:
    """agents/agents.py:10-28."""
    actor_net: tuple
    actor_learning_rate: float
    critic_net: tuple
    critic_learning_rate: float
    optimizer: str
    max_grad_norm: float
    critic_dims: int = 1

    @staticmethod
    def from_args(args):
        h = get_agent_hypers(args.env_mode)
        return AgentHyperparams(**h, critic_dims=args.lpg_target_width)

    def check_supported(self):
        if self.actor_net or self.critic_net or self.optimizer != "SGD":
            raise NotImplementedError(
                "MI355X hot path implements the tabular agents (actor_net=(), SGD with global-norm clip) used by "
                "every BASELINE config; MLP agents with Adam (rand_* modes) are out of scope (DESIGN.md)")


def lecun_tables(keys: torch.Tensor, D: int, cols: int) -> torch.Tensor:
    """flax lecun_normal Dense(cols, use_bias=False) kernels [n, D, cols], one per key."""
    n = keys.shape[0]
    out = torch.empty((n, D, cols), dtype=torch.float32, device=keys.device)
    std = math.sqrt(1.0 / D) / 0.87962566103423978
    _lib.call("toued_init_tables", _lib.ptr(keys.contiguous()), n, cols, D, TN_LO, TN_HI, std, _lib.ptr(out),
              _lib.stream_ptr())
    return out


def create_agents(agent_keys: torch.Tensor, D: int, Y: int):
    """create_agent (agents/agents.py:31-56) for each key: actor_rng, critic_rng = split(agent_rng)."""
    ks = prng.split(agent_keys, 2)
    theta = lecun_tables(ks[:, 0].contiguous(), D, 5)
    phi = lecun_tables(ks[:, 1].contiguous(), D, Y)
    return theta, phi


def create_value_critics(keys: torch.Tensor, D: int) -> torch.Tensor:
    """create_value_critic (agents/agents.py:59-75): Dense(1) kernels [n, D]."""
    return lecun_tables(keys, D, 1).reshape(keys.shape[0], D)


@dataclass
class AgentBatch:
    levels: torch.Tensor
    theta: torch.Tensor
    phi: torch.Tensor
    step: torch.Tensor
    state: torch.Tensor
    vcrit: torch.Tensor | None = None
    vstep: torch.Tensor | None = None

    @property
    def n(self) -> int:
        return self.levels.shape[0]
