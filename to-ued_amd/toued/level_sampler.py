"""UED level sampler on MI355X (environments/level_sampler.py:30-416).

``LevelSampler(args)`` mirrors the reference: ``initialize_buffer``,
``initial_sample``, ``sample``, ``rollout_manager``, ``max_lifetime``.
Score functions: ``random`` (domain randomisation), ``frozen`` (uniform replay
of a fixed buffer) and ``alg_regret`` (PLR with the A2C antagonist's
algorithmic regret, GROOVE).  All state is device-resident; per-agent work is
computed for the whole batch and masked by ``terminated`` exactly like the
reference's vmapped ``jnp.where`` (the masked-out work has no observable effect).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib, prng
from .agents import (DENSE0_HASH, AgentBatch, AgentHyperparams, create_agents, create_agents_into,
                     create_value_critics, lecun_tables_into, lecun_tables_into_folded)
from .env import L_BUFID, L_LIFETIME, LevelGenerator, get_env_spec
from .rollout import RolloutWrapper

SCORE_FUNCTIONS = ["random", "frozen", "alg_regret"]
SCORE_TRANSFORMS = ["proportional", "rank"]


@dataclass
class LevelBuffer:
    """level_sampler.py:30-52: packed levels [B,64] (buffer_id packed), score, active, new."""
    levels: torch.Tensor
    score: torch.Tensor
    active: torch.Tensor
    new: torch.Tensor

    def __len__(self):
        return self.score.shape[0]


def cumsum_assoc_np(p: np.ndarray) -> np.ndarray:
    """jnp.cumsum as lowered by jax 0.4.13 on CPU (lax.associative_scan order), float32."""
    p = np.asarray(p, np.float32)

    def scan(e):
        n = e.shape[-1]
        if n < 2:
            return e
        odd = scan(e[0:-1:2] + e[1::2])
        even = (odd[:-1] + e[2::2]) if n % 2 == 0 else (odd + e[2::2])
        even = np.concatenate([e[0:1], even])
        out = np.empty_like(e)
        out[0::2] = even
        out[1::2] = odd
        return out

    return scan(p)


class LevelSampler:
    def __init__(self, args, device=None, world=None):
        self.env_name = args.env_name
        self.env_mode = args.env_mode
        self.env_workers = args.env_workers
        self.spec, self.max_rollout_len, self.max_lifetime = get_env_spec(self.env_mode)
        self.rollout_manager = RolloutWrapper(self.env_mode, args.train_rollout_len, self.max_rollout_len,
                                              args.env_workers)
        self.agent_hypers = AgentHyperparams.from_args(args)
        self.agent_hypers.check_supported()
        if args.score_function not in SCORE_FUNCTIONS:
            raise ValueError(f"Level score function {args.score_function} not in known functions: {SCORE_FUNCTIONS}")
        if args.score_transform not in SCORE_TRANSFORMS:
            raise ValueError(
                f"Level score transform {args.score_transform} not in known transforms: {SCORE_TRANSFORMS}")
        self.score_function = args.score_function
        self.score_transform = args.score_transform
        self.score_temperature = args.score_temperature
        self.buffer_size = args.buffer_size
        self.p_replay = args.p_replay
        self.num_mini_batches = args.num_mini_batches
        self.args = args
        self.world = world
        self.dev = torch.device(device) if device is not None else torch.device("cuda")
        self.gen = LevelGenerator(self.env_mode, self.dev)
        self.Y = args.lpg_target_width
        self._cdf = None
        self.regret_all_agents = bool(getattr(args, "regret_all_agents", False))
        self._a2c = None
        self.last_plr = None

    def a2c_trainer(self):
        """The A2C antagonist trainer (level_sampler.py:86-88, 296-310), built on first use."""
        if self._a2c is None:
            from .a2c import A2CHyperparams, A2CTrainer
            self._a2c = A2CTrainer(self.rollout_manager,
                                   A2CHyperparams(self.args.gamma, self.args.gae_lambda, self.args.entropy_coeff),
                                   self.agent_hypers)
        return self._a2c

    @property
    def obs_dim(self) -> int:
        return self.spec.obs_dim

    @property
    def num_actions(self) -> int:
        return 5

    # ------------------------------------------------------------------ helpers
    def _slice(self, x: torch.Tensor, sl):
        return x if sl is None else x[sl[0]:sl[1]].contiguous()

    def _sample_random_levels(self, rng, n_total, sl):
        """level_sampler.py:268-271: split(rng, N) -> reset_env_params; buffer_id = 0."""
        keys = self._slice(prng.split(rng, n_total), sl)
        return self.gen(keys)

    def _create_agents(self, rng, levels, n_total, sl, create_value_critics_too: bool):
        """vmap(_create_agent) (level_sampler.py:273-291): worker_rng, agent_rng = split(rng_i)."""
        keys = self._slice(prng.split(rng, n_total), sl)
        ks = prng.split_planar(keys, 2)    # ks[j] = split(keys, 2)[:, j], contiguous
        (_, _), state = self.rollout_manager.batch_reset(ks[0], levels)
        theta, phi = create_agents(ks[1], self.obs_dim, self.Y)
        return theta, phi, state

    # ------------------------------------------------------------------ API
    def initialize_buffer(self, rng):
        """level_sampler.py:90-96 (None for score_function=random)."""
        if self.score_function == "random":
            return None
        keys = prng.split(rng, self.buffer_size)
        ids = torch.arange(self.buffer_size, dtype=torch.int32, device=self.dev)
        levels = self.gen(keys, buffer_ids=ids)
        B = self.buffer_size
        return LevelBuffer(levels, torch.zeros(B, device=self.dev), torch.zeros(B, dtype=torch.bool, device=self.dev),
                           torch.ones(B, dtype=torch.bool, device=self.dev))

    def initial_sample(self, rng, level_buffer, batch_size: int, create_value_critics_flag: bool, sl=None):
        """level_sampler.py:103-132.  ``sl`` = (lo, hi, total) agent slice of this rank."""
        n_local = batch_size if sl is None else sl[1] - sl[0]
        if self.score_function == "random":
            # only the random branch splits here (level_sampler.py:112-114); the buffer branch does not
            rng, sub = self._split2(rng)
            levels = self._sample_random_levels(sub, batch_size, sl)
        else:
            levels = self._slice(level_buffer.levels[:batch_size], sl)
            level_buffer.active = torch.arange(self.buffer_size, device=self.dev) < batch_size
        rng, sub = self._split2(rng)
        theta, phi, state = self._create_agents(sub, levels, batch_size, sl, False)
        vcrit = None
        if create_value_critics_flag:
            rng, sub = self._split2(rng)
            vcrit = create_value_critics(self._slice(prng.split(sub, batch_size), sl), self.obs_dim)
        agents = AgentBatch(levels, theta, phi, torch.zeros(n_local, dtype=torch.int32, device=self.dev), state,
                            vcrit, torch.zeros(n_local, dtype=torch.int32, device=self.dev) if vcrit is not None
                            else None)
        return level_buffer, agents

    @staticmethod
    def _split2(rng):
        ks = prng.split_planar(rng.view(1, 2), 2)
        return ks[0, 0], ks[1, 0]

    def sample(self, rng, level_buffer, agents: AgentBatch, sl=None):
        """level_sampler.py:134-266: new levels/agents for agents whose step >= lifetime.

        The reference builds a full batch of new levels/agents/env states and keeps the terminated agents'
        (``where(term, new, old)``); here the generators write the terminated agents' rows in place (same
        keys, same values) and leave the others untouched."""
        n_total = agents.n if sl is None else sl[2]
        if self.score_function == "random" and os.environ.get("TOUED_SAMPLE_FUSED", "1") != "0":
            return level_buffer, self._sample_random_fused(rng, agents, n_total, 0 if sl is None else sl[0])
        term = agents.step >= agents.levels[:, L_LIFETIME]
        mask = term.to(torch.uint8)
        if self.score_function == "random":
            rng, sub = self._split2(rng)
            self.gen.regenerate(self._slice(prng.split(sub, n_total), sl), agents.levels, mask)
        else:
            if self.score_function == "frozen":
                rng, sub = self._split2(rng)
                ids = self._frozen_ids(sub, n_total)
                new_levels = self._slice(level_buffer.levels[ids.long()], sl)
            else:
                from .plr import plr_sample
                rng, level_buffer, new_levels = plr_sample(self, rng, level_buffer, agents, term, sl)
            agents.levels = torch.where(term[:, None], new_levels, agents.levels)
        # vmap(_create_agent) (level_sampler.py:273-291): worker_rng, agent_rng = split(rng_i)
        rng, sub = self._split2(rng)
        ks = prng.split_planar(self._slice(prng.split(sub, n_total), sl), 2)
        self.rollout_manager.batch_reset_into(ks[0], agents.levels, agents.state, mask)
        create_agents_into(ks[1], agents.theta, agents.phi, mask)
        agents.step = torch.where(term, torch.zeros_like(agents.step), agents.step)
        if agents.vcrit is not None:
            rng, sub = self._split2(rng)
            n = agents.vcrit.shape[0]
            lecun_tables_into(self._slice(prng.split(sub, n_total), sl), agents.vcrit.view(n, self.obs_dim, 1), mask)
            agents.vstep = torch.where(term, torch.zeros_like(agents.vstep), agents.vstep)
        return level_buffer, agents

    def _sample_random_fused(self, rng, agents: AgentBatch, n_total: int, lo: int) -> AgentBatch:
        """The random branch of ``sample`` with its termination test and key derivations in one launch
        (toued_sample_random_keys: the same keys and masks as the split / fold_in chain below, bit-identical), then
        the masked level generator, env reset and table inits; step / vstep are zeroed in place where terminated.
        TOUED_SAMPLE_FUSED=0 takes the launch-per-operation path."""
        n = agents.n
        nk = 5 if agents.vcrit is not None else 4
        if getattr(self, "_rk", None) is None or self._rk[0].shape != (nk, n, 2):
            self._rk = (torch.empty((nk, n, 2), dtype=torch.int32, device=self.dev),
                        torch.empty((n,), dtype=torch.uint8, device=self.dev))
        keys, mask = self._rk
        vstep = agents.vstep if agents.vcrit is not None else None
        _lib.call("toued_sample_random_keys", _lib.ptr(rng.contiguous()), n_total, lo, n, _lib.ptr(agents.step),
                  _lib.ptr(agents.levels), _lib.ptr(vstep), DENSE0_HASH, _lib.ptr(mask), _lib.ptr(keys),
                  _lib.stream_ptr())
        self.gen.regenerate(keys[0], agents.levels, mask)
        self.rollout_manager.batch_reset_into(keys[1], agents.levels, agents.state, mask)
        lecun_tables_into_folded(keys[2], agents.theta, mask)
        lecun_tables_into_folded(keys[3], agents.phi, mask)
        if agents.vcrit is not None:
            lecun_tables_into_folded(keys[4], agents.vcrit.view(n, self.obs_dim, 1), mask)
        return agents

    def _frozen_ids(self, rng, n):
        """random.choice(arange(B), p=uniform, shape=(N,), replace=True) (level_sampler.py:157-165)."""
        if self._cdf is None:
            c = cumsum_assoc_np(np.full(self.buffer_size, np.float32(1.0) / np.float32(self.buffer_size), np.float32))
            self._cdf = torch.from_numpy(c).to(self.dev)
        out = torch.empty(n, dtype=torch.int32, device=self.dev)
        _lib.call("toued_choice_cdf", _lib.ptr(rng.contiguous()), _lib.ptr(self._cdf), self.buffer_size, n,
                  _lib.ptr(out), _lib.stream_ptr())
        return out
