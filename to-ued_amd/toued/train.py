"""Meta-training driver (train.py:14-82 of the reference) on MI355X.

    python -m toued.train --env_mode tabular --num_agents 512 --num_mini_batches 1 [--score_function alg_regret]
                         [--use_es --lifetime_conditioning] [--train_steps N | --ref_quirk_steps10]

One process per GPU (torchrun): agents are sharded over ranks; the LPG
parameters are replicated and updated identically on every rank after the
meta-gradient all-reduce.  ``--num_mini_batches`` splits each rank's agents into
that many sequential chunks for the meta-gradient (util/jax.py:25-41
mini_batch_vmap: numerically a no-op, a memory bound); 1 runs the whole batch at
once, which 288 GB of HBM holds up to ~620 agents per GPU at W=64, T=20, K=5.
"""
from __future__ import annotations

import json
import sys
import time

import numpy as np
import torch

from . import _lib, prng
from .debug import configure as configure_debug
from .dist import World, init_from_env
from .level_sampler import LevelSampler
from .lpg import flax_init_lpg_params
from .meta import (AdamState, LpgTrainState, MetaGradStep, lpg_hypers_from_args,  # noqa: F401 (re-exported)
                   make_lpg_train_step)
from .parse_args import parse_args


def check_supported(args):
    if args.env_name != "GridWorld-v0":
        raise NotImplementedError("gymnax environments are out of scope (DESIGN.md); use GridWorld-v0")
    if (args.lpg_gru_width, args.lpg_target_width, args.lpg_embedding_net_width) != (256, 8, 16):
        raise NotImplementedError("the MFMA LPG kernels are built for gru_width=256, target_width=8, embedding=16")
    if args.lpg_opt.lower() != "adam" and not args.use_es:
        raise NotImplementedError("meta-gradient LPG optimiser: Adam (models/optim.py:12-17)")


class Trainer:
    """make_train(args) (train.py:14-59) as a stateful object with one method per meta-step."""

    def __init__(self, args, world: World | None = None, device=None):
        check_supported(args)
        self.args = args
        # util/jax.py:5-17: --debug_nans raises at the first non-finite stage, --debug checks every call synchronously
        self.nans = configure_debug(debug=getattr(args, "debug", False), debug_nans=getattr(args, "debug_nans", False))
        self.world = world or World()
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        sl = self.world.agent_slice(args.num_agents) if self.world.size > 1 else None
        self.sl = sl
        rng = prng.PRNGKey(args.seed, self.dev)
        ks = prng.split(rng, 3)
        self.rng, lpg_rng, buffer_rng = ks[0].contiguous(), ks[1].contiguous(), ks[2].contiguous()
        F = 7 if args.lifetime_conditioning else 5
        # create_lpg_train_state (meta/meta.py:21-22): flax's init of the LPG from lpg_rng
        self.eta = flax_init_lpg_params(lpg_rng, F)
        self.eta_init = self.eta.clone()
        self.sampler = LevelSampler(args, self.dev, self.world)
        self.buffer = self.sampler.initialize_buffer(buffer_rng)
        ks = prng.split(self.rng, 2)
        self.rng, sub = ks[0].contiguous(), ks[1].contiguous()
        n_local = args.num_agents if sl is None else sl[1] - sl[0]
        self.buffer, self.agents = self.sampler.initial_sample(sub, self.buffer, args.num_agents,
                                                               not args.use_es, sl)
        self.buffer_init = None
        if self.buffer is not None and getattr(args, "ref_quirk_checkpoint_init", False):
            from .level_sampler import LevelBuffer
            b = self.buffer
            self.buffer_init = LevelBuffer(b.levels.clone(), b.score.clone(), b.active.clone(), b.new.clone())
        if args.use_es:
            from .es import ESTrainStep
            self.step_fn = ESTrainStep(args, self.sampler, n_local, self.eta, self.dev, self.world)
        else:
            self.hyp = lpg_hypers_from_args(args, self.sampler)
            self.step_fn = MetaGradStep(self.sampler.rollout_manager, n_local, self.hyp, args.lifetime_conditioning,
                                        self.dev, self.world, num_mini_batches=args.num_mini_batches,
                                        num_agents_global=args.num_agents)
            self.adam = AdamState(self.eta.numel(), self.dev)
        # the reference's lpg_train_step_fn (train.py:33, meta/meta.py:33-52) driving this instance
        self.train_state = LpgTrainState(self.eta, None if args.use_es else self.adam)
        self.train_step = make_lpg_train_step(args, self.sampler, n_local, self.world, sl, impl=self.step_fn)

    def meta_step(self):
        """_meta_train_loop (train.py:36-54): LPG update, then level_sampler.sample."""
        # split(rng) with the key axis first: both halves contiguous, no copy launches
        ks = prng.split_planar(self.rng.view(1, 2), 2)
        self.rng, sub = ks[0, 0], ks[1, 0]
        self.train_state, self.agents, _, metrics = self.train_step(sub, self.train_state, self.agents)
        ks = prng.split_planar(self.rng.view(1, 2), 2)
        self.rng, sub = ks[0, 0], ks[1, 0]
        self.buffer, self.agents = self.sampler.sample(sub, self.buffer, self.agents, self.sl)
        self.nans.raise_if_any()
        return metrics

    def finish(self):
        """End of training: report any device error a round left behind (synchronising once)."""
        _lib.check_device_errors(wait=True)


def reduce_metrics(m, world: World):
    """Mean over agents (meta/train.py:180), across ranks when distributed."""
    if isinstance(m, dict):
        return {k: reduce_metrics(v, world) for k, v in m.items()}
    if not torch.is_tensor(m):
        return m
    if m.dim() == 0:
        return float(m)
    s = m.float().sum().reshape(1)
    n = torch.tensor([m.numel()], dtype=torch.float32, device=m.device)
    world.all_reduce_sum(s)
    world.all_reduce_sum(n)
    return float(s / n)


def main(cmd_args=None):
    args = parse_args(cmd_args)
    world = init_from_env()
    tr = Trainer(args, world)
    steps = 10 if args.ref_quirk_steps10 else args.train_steps
    history = []
    t0 = time.time()
    for i in range(steps):
        m = reduce_metrics(tr.meta_step(), world)
        history.append(m)
        if world.rank == 0:
            print(json.dumps({"step": i, "elapsed_s": round(time.time() - t0, 3), **m}), flush=True)
    tr.finish()
    if args.checkpoint_dir and world.rank == 0:
        save_final_checkpoints(args.checkpoint_dir, tr, steps)
    return history


def save_final_checkpoints(ckpt_dir: str, tr: "Trainer", steps: int):
    """log_results (experiments/logging.py:31-46) without wandb: the LPG train state as checkpoint_<steps> and, for
    buffer-based score functions, the level buffer as buffer_checkpoint_<steps> (toued/checkpoint.py), both in the
    reference's pytree layouts.  With --ref_quirk_checkpoint_init the states written are the ones the reference's
    _train_fn actually returns -- the initial train state and level buffer, because the scan's final carry is never
    unpacked (train.py:52-57) -- instead of the trained ones."""
    from .checkpoint import es_train_state_dict, level_buffer_state_dict, lpg_train_state_dict, save_checkpoint
    from .lpg import LPGLayout
    lay = LPGLayout(7 if tr.args.lifetime_conditioning else 5)
    init = bool(getattr(tr.args, "ref_quirk_checkpoint_init", False))
    if tr.args.use_es:
        es = tr.step_fn.es
        if init:
            from .es import OpenES
            a = tr.args
            es = OpenES(es.popsize, es.nd, a.lpg_opt, a.lpg_learning_rate, a.es_lrate_decay, a.es_lrate_limit,
                        a.es_sigma_init, a.es_sigma_decay, a.es_sigma_limit, a.es_mean_decay, tr.dev)
        target = es_train_state_dict(es, tr.eta_init, lay, tr.args.lpg_opt, es.best_member, es.best_fitness)
    elif init:
        target = lpg_train_state_dict(tr.eta_init, lay, 0, None)
    else:
        target = lpg_train_state_dict(tr.eta, lay, steps, tr.adam)
    save_checkpoint(ckpt_dir, target, steps)
    buf = tr.buffer_init if init else tr.buffer
    if buf is not None:
        save_checkpoint(ckpt_dir, level_buffer_state_dict(buf, tr.sampler.spec), steps, prefix="buffer_")


if __name__ == "__main__":
    main(sys.argv[1:])
