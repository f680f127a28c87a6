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

import hashlib
import math
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib, prng
from .env import get_agent_hypers

# lax.erf(-+2 / sqrt2) in float32 (XLA's f32 erf; equals the correctly rounded value here)
TN_LO = -0.9544997215270996
TN_HI = 0.9544997215270996


def flax_static_hash(path) -> int:
    """flax 0.6.11 param-key derivation (core/scope.py, lazy RNG): ``self.param`` draws with
    fold_in(rng, h) where h = the first 4 bytes (big-endian) of sha1 over the module path names and the
    scope's 'params' counter (minimal big-endian bytes), hashed together without separators."""
    m = hashlib.sha1()
    for x in path:
        m.update(x.encode("utf-8") if isinstance(x, str) else x.to_bytes((x.bit_length() + 7) // 8, "big"))
    return int.from_bytes(m.digest()[:4], "big")


# the kernel of Actor / Critic's inline Dense (models/agent.py:7-45, actor_net=()): path Dense_0, counter 1
DENSE0_HASH = flax_static_hash(("Dense_0", 1))


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
    """``model.init(key, obs)`` of Actor/Critic with actor_net=() (models/agent.py:7-45): the
    Dense(cols, use_bias=False) kernel, flax lecun_normal = truncated_normal(-2, 2) * stddev with
    stddev = sqrt(1/D) / .87962566103423978 in float32.  Returns [n, D, cols], one per key."""
    n = keys.shape[0]
    out = torch.empty((n, D, cols), dtype=torch.float32, device=keys.device)
    pkeys = prng.fold_in(keys.contiguous(), DENSE0_HASH)
    std = float(np.float32(np.sqrt(np.float32(1.0 / D))) / np.float32(0.87962566103423978))
    _lib.call("toued_init_tables", _lib.ptr(pkeys.contiguous()), n, cols, D, TN_LO, TN_HI, std, _lib.ptr(out),
              _lib.stream_ptr())
    return out


def lecun_tables_into(keys: torch.Tensor, out: torch.Tensor, mask: torch.Tensor):
    """``lecun_tables(keys, D, cols)`` written in place into ``out`` [n, D, cols] for the tables with
    ``mask`` (u8 [n]) set; the others keep their values (the level sampler's where(terminated, new, old))."""
    n, D, cols = out.shape
    pkeys = prng.fold_in(keys.contiguous(), DENSE0_HASH)
    std = float(np.float32(np.sqrt(np.float32(1.0 / D))) / np.float32(0.87962566103423978))
    _lib.call("toued_init_tables_masked", _lib.ptr(pkeys.contiguous()), n, cols, D, TN_LO, TN_HI, std, _lib.ptr(out),
              _lib.ptr(mask), _lib.stream_ptr())
    return out


def lecun_tables_into_folded(pkeys: torch.Tensor, out: torch.Tensor, mask: torch.Tensor):
    """``lecun_tables_into`` with the keys already folded with DENSE0_HASH (toued_sample_random_keys)."""
    n, D, cols = out.shape
    std = float(np.float32(np.sqrt(np.float32(1.0 / D))) / np.float32(0.87962566103423978))
    _lib.call("toued_init_tables_masked", _lib.ptr(pkeys), n, cols, D, TN_LO, TN_HI, std, _lib.ptr(out),
              _lib.ptr(mask), _lib.stream_ptr())
    return out


def create_agents_into(agent_keys: torch.Tensor, theta: torch.Tensor, phi: torch.Tensor, mask: torch.Tensor):
    """``create_agents`` for the agents with ``mask`` set, in place into theta [n, D, 5] / phi [n, D, Y]."""
    ks = prng.split_planar(agent_keys, 2)   # ks[j] = split(agent_keys, 2)[:, j], contiguous
    lecun_tables_into(ks[0], theta, mask)
    lecun_tables_into(ks[1], phi, mask)


def create_agents(agent_keys: torch.Tensor, D: int, Y: int):
    """create_agent (agents/agents.py:31-56) for each key: actor_rng, critic_rng = split(agent_rng)."""
    ks = prng.split_planar(agent_keys, 2)
    theta = lecun_tables(ks[0], D, 5)
    phi = lecun_tables(ks[1], D, Y)
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


def eval_agent(ro, rng: torch.Tensor, levels: torch.Tensor, theta: torch.Tensor, num_workers: int) -> torch.Tensor:
    """agents/agents.py:98-106 for n agents: (rng, _rng) = split(rng) -> batch_reset(_rng, W);
    (rng, _rng) = split(rng) -> eval rollout; mean first-episode return per agent, f32 [n]."""
    state, keys = eval_agent_reset(ro, rng, levels, num_workers)
    return ro.eval_returns(keys, theta, levels, state).mean(dim=1)


def eval_agent_reset(ro, rng: torch.Tensor, levels: torch.Tensor, num_workers: int):
    """eval_agent's table-independent part: the worker reset and the rollout keys (agents/agents.py:100-103).
    Returns (state [12, n*W], rollout keys [n, 2]) for RolloutWrapper.eval_returns(keys, theta, levels, state) or,
    through RolloutWrapper.eval_draws(keys, levels, W), eval_returns_from_draws."""
    ks = prng.split_planar(rng, 2)     # ks[j] = split(rng, 2)[:, j], contiguous
    (_, _), state = ro.batch_reset(ks[1], levels, num_workers)
    return state, prng.split_planar(ks[0], 2)[1]
