"""RolloutWrapper on MI355X (environments/rollout.py:13-102), vmapped over agents.

The reference's ``RolloutWrapper`` works on one agent and is vmapped by its
callers (agents/a2c.py:98, agents/lpg_agent.py:109, meta/train.py:48,
agents/agents.py:101-105, level_sampler.py:276).  Here the agent axis is
explicit: every call takes N agent keys, N packed levels and N actor tables,
and runs one fused HIP launch (csrc/env.hip k_rollout).  Called with the reference's
single-agent arguments instead -- one key ``rng`` of shape [2], one level, one actor table
``[D, 5]`` -- ``batch_reset``/``batch_rollout`` run that one agent and return its results
without the agent axis, as ``RolloutWrapper.batch_reset(rng, env_params, num_workers)`` and
``batch_rollout(rng, train_state, env_params, init_obs, init_state)`` do.
"""
from __future__ import annotations

import os

from dataclasses import dataclass

import torch

from . import _lib
from .env import STATE_FIELDS, EnvSpec, get_env_spec


@dataclass
class Transition:
    """util/data.py:37-44 in compact, lane-contiguous layout.

    obs_idx/obs_time: int32 [N, T+1, W] (obs_t for t<T; slot T is the end obs,
    so next_obs_t == obs_{t+1}); action/done: uint8 [N, T, W]; reward: f32 [N, T, W].
    """
    obs_idx: torch.Tensor
    obs_time: torch.Tensor
    action: torch.Tensor
    reward: torch.Tensor
    done: torch.Tensor


def split_rollouts() -> bool:
    """Train rollouts as draws + env chain (toued_rollout_draws / toued_rollout_env) unless TOUED_ROLLOUT_FUSED=1
    (the single-kernel toued_rollout; bit-identical)."""
    return os.environ.get("TOUED_ROLLOUT_FUSED") != "1"


class RolloutWrapper:
    def __init__(self, env_mode: str, train_rollout_len: int, eval_rollout_len: int | None = None,
                 env_workers: int = 64):
        self.env_mode = env_mode
        self.spec, max_len, _ = get_env_spec(env_mode)
        self.train_rollout_len = train_rollout_len
        self.eval_rollout_len = max_len if eval_rollout_len is None else eval_rollout_len
        self.env_workers = env_workers
        self._c = _lib.env_spec_c(self.spec)

    @property
    def obs_dim(self) -> int:
        return self.spec.obs_dim

    def batch_reset(self, agent_keys: torch.Tensor, levels: torch.Tensor, num_workers: int | None = None):
        """rollout.py:38-42 per agent: split(rng, W); vmap(env.reset).  Returns ((idx, time) [N*W], state).
        A single key [2] and level resets that one agent's W workers (the reference's unvmapped call)."""
        if agent_keys.dim() == 1:
            return self.batch_reset(agent_keys.view(1, 2), levels.view(1, -1), num_workers)
        W = self.env_workers if num_workers is None else num_workers
        N = agent_keys.shape[0]
        dev = agent_keys.device
        n = N * W
        # zeroed: the kernel writes the mode's fields only (object slots past max_n_objs stay 0, not stale memory)
        state = torch.zeros((STATE_FIELDS, n), dtype=torch.int32, device=dev)
        idx = torch.empty(n, dtype=torch.int32, device=dev)
        tm = torch.empty(n, dtype=torch.int32, device=dev)
        _lib.call("toued_batch_reset", self._c, _lib.ptr(levels), _lib.ptr(agent_keys.contiguous()), N, W,
                  _lib.ptr(state), _lib.ptr(idx), _lib.ptr(tm), _lib.stream_ptr())
        return (idx, tm), state

    def batch_reset_into(self, agent_keys: torch.Tensor, levels: torch.Tensor, state: torch.Tensor,
                         mask: torch.Tensor):
        """``batch_reset`` in place into ``state`` [fields, N*W] for the agents with ``mask`` (u8 [N]) set."""
        N = agent_keys.shape[0]
        W = state.shape[1] // N
        n = N * W
        if getattr(self, "_obs_scratch", None) is None or self._obs_scratch.shape[1] < n:
            self._obs_scratch = torch.empty((2, n), dtype=torch.int32, device=state.device)
        _lib.call("toued_batch_reset_masked", self._c, _lib.ptr(levels), _lib.ptr(agent_keys.contiguous()), N, W,
                  _lib.ptr(state), _lib.ptr(self._obs_scratch[0]), _lib.ptr(self._obs_scratch[1]), _lib.ptr(mask),
                  _lib.stream_ptr())
        return state

    def batch_rollout(self, agent_keys: torch.Tensor, theta: torch.Tensor, levels: torch.Tensor,
                      state: torch.Tensor, eval: bool = False, out: Transition | None = None,
                      inplace_state: bool = False):
        """rollout.py:45-102.  theta: actor tables f32 [N, D, 5].

        Returns (Transition, end_state, cum_return f32 [N, W]).  With a single key [2] (one level, theta [D, 5]):
        the reference's single-agent batch_rollout, results without the agent axis (cum_return [W]).
        """
        if agent_keys.dim() == 1:
            o = None if out is None else Transition(*(x.unsqueeze(0) for x in (out.obs_idx, out.obs_time, out.action,
                                                                              out.reward, out.done)))
            tr, st, cum = self.batch_rollout(agent_keys.view(1, 2), theta.unsqueeze(0), levels.view(1, -1), state,
                                             eval=eval, out=o, inplace_state=inplace_state)
            return Transition(tr.obs_idx[0], tr.obs_time[0], tr.action[0], tr.reward[0], tr.done[0]), st, cum[0]
        N = agent_keys.shape[0]
        n = state.shape[1]
        W = n // N
        T = self.eval_rollout_len if eval else self.train_rollout_len
        D = theta.shape[1]
        dev = state.device
        if not inplace_state:
            state = state.clone()
        if out is None:
            out = Transition(
                torch.empty((N, T + 1, W), dtype=torch.int32, device=dev),
                torch.empty((N, T + 1, W), dtype=torch.int32, device=dev),
                torch.empty((N, T, W), dtype=torch.uint8, device=dev),
                torch.empty((N, T, W), dtype=torch.float32, device=dev),
                torch.empty((N, T, W), dtype=torch.uint8, device=dev),
            )
        cum = torch.empty((N, W), dtype=torch.float32, device=dev)
        if eval or not split_rollouts():
            _lib.call("toued_rollout", self._c, _lib.ptr(levels), _lib.ptr(theta), D,
                      _lib.ptr(agent_keys.contiguous()), _lib.ptr(state), N, W, T, _lib.ptr(out.obs_idx),
                      _lib.ptr(out.obs_time), _lib.ptr(out.action), _lib.ptr(out.reward), _lib.ptr(out.done),
                      _lib.ptr(cum), _lib.stream_ptr())
            return out, state, cum
        draws = self.train_draws(agent_keys.view(1, N, 2), levels, W)
        self.rollout_from_draws(draws, 0, theta, levels, state, out, cum)
        return out, state, cum

    def train_draws(self, keys: torch.Tensor, levels: torch.Tensor, n_workers: int,
                    bufs: tuple[torch.Tensor, torch.Tensor] | None = None, stream: int | None = None) -> torch.Tensor:
        """The state-independent draws of U batches of train rollouts (toued_rollout_draws): keys [U, N, 2] (batch u's
        rollout keys), levels [N, words].  Returns u32 [T, U * N * W, 4]: in ``bufs`` = (chain scratch, draws), each
        at least [T, U * N * W, 4] (the step stride is theirs), or in a buffer of this wrapper reused by the next
        call of the same shape.  ``stream``: a raw HIP stream to launch on (default: torch's current stream)."""
        U, N = keys.shape[0], keys.shape[1]
        T, W = self.train_rollout_len, n_workers
        n = U * N * W
        if bufs is not None:
            chain, draws = bufs
            if chain.shape[0] < T or chain.shape[1] < n or draws.shape != chain.shape:
                raise ValueError(f"train_draws: buffers {tuple(chain.shape)} for T={T}, {n} workers")
            n = chain.shape[1]
        else:
            key = (T, n, str(levels.device))
            if getattr(self, "_draw_bufs", None) is None or self._draw_bufs[0] != key:
                self._draw_bufs = (key, torch.empty((T, n, 4), dtype=torch.int32, device=levels.device),
                                   torch.empty((T, n, 4), dtype=torch.int32, device=levels.device))
            _, chain, draws = self._draw_bufs
        if n != U * N * W:
            raise ValueError("train_draws: the buffers' worker stride must equal U * N * W")
        _lib.call("toued_rollout_draws", self._c, _lib.ptr(levels), _lib.ptr(keys.contiguous()), N, U, W, T,
                  _lib.ptr(chain), _lib.ptr(draws), stream if stream is not None else _lib.stream_ptr())
        return draws

    def rollout_from_draws(self, draws: torch.Tensor, u: int, theta: torch.Tensor, levels: torch.Tensor,
                           state: torch.Tensor, out: Transition, cum: torch.Tensor | None = None):
        """Batch u of train_draws' rollouts (toued_rollout_env): trajectories into ``out``, ``state`` advanced in place;
        bit-identical to toued_rollout with the same keys."""
        N = theta.shape[0]
        n = state.shape[1]
        T = self.train_rollout_len
        _lib.call("toued_rollout_env", self._c, _lib.ptr(levels), _lib.ptr(theta), theta.shape[1], _lib.ptr(state), N,
                  n // N, T, _lib.ptr(draws) + 16 * u * n, draws.shape[1], _lib.ptr(out.obs_idx),
                  _lib.ptr(out.obs_time), _lib.ptr(out.action), _lib.ptr(out.reward), _lib.ptr(out.done),
                  _lib.ptr(cum) if cum is not None else None, _lib.stream_ptr())

    def eval_draws(self, agent_keys: torch.Tensor, levels: torch.Tensor, n_workers: int,
                   buf: torch.Tensor | None = None) -> torch.Tensor:
        """The state-independent draws of an eval-length returns-only rollout (toued_eval_keys, toued_eval_draws):
        u32 [T, N*W, 4], consumed by eval_returns_from_draws.  They depend on the keys and levels only, so they can
        be produced early, beside other work."""
        N = agent_keys.shape[0]
        n, T = N * n_workers, self.eval_rollout_len
        dev = levels.device
        chain = torch.empty((T, n, 4), dtype=torch.int32, device=dev)
        if buf is None or buf.shape != (T, n, 4):
            buf = torch.empty((T, n, 4), dtype=torch.int32, device=dev)
        st = _lib.stream_ptr()
        _lib.call("toued_eval_keys", _lib.ptr(agent_keys.contiguous()), N, n_workers, T, _lib.ptr(chain), st)
        _lib.call("toued_eval_draws", self._c, _lib.ptr(levels), N, n_workers, T, _lib.ptr(chain), _lib.ptr(buf), st)
        return buf

    def eval_returns_from_draws(self, draws: torch.Tensor, theta: torch.Tensor, levels: torch.Tensor,
                                state: torch.Tensor) -> torch.Tensor:
        """eval_returns on draws from eval_draws (same keys, levels and worker count): bit-identical.
        Returns f32 [N, W]."""
        N = theta.shape[0]
        n = state.shape[1]
        cum = torch.empty((N, n // N), dtype=torch.float32, device=state.device)
        _lib.call("toued_eval_returns", self._c, _lib.ptr(levels), _lib.ptr(theta), theta.shape[1], _lib.ptr(state),
                  N, n // N, self.eval_rollout_len, _lib.ptr(draws), _lib.ptr(cum), _lib.stream_ptr())
        return cum

    def eval_returns(self, agent_keys: torch.Tensor, theta: torch.Tensor, levels: torch.Tensor,
                     state: torch.Tensor) -> torch.Tensor:
        """batch_rollout(..., eval=True) when only cum_return is consumed (eval_agent): returns-only
        kernel mode, no trajectory stores; `state` is left unmodified.  Returns f32 [N, W]."""
        N = agent_keys.shape[0]
        n = state.shape[1]
        cum = torch.empty((N, n // N), dtype=torch.float32, device=state.device)
        _lib.call("toued_rollout", self._c, _lib.ptr(levels), _lib.ptr(theta), theta.shape[1],
                  _lib.ptr(agent_keys.contiguous()), _lib.ptr(state), N, n // N, self.eval_rollout_len, None, None,
                  None, None, None, _lib.ptr(cum), _lib.stream_ptr())
        return cum
