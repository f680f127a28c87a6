"""PLR / GROOVE level scoring on MI355X (environments/level_sampler.py:169-234, 293-408).

``plr_sample`` is the ``alg_regret`` branch of ``LevelSampler.sample``:
  1. ``_reset_lowest_scoring`` (:331-353): toued_plr_reset_ids (LDS bitonic argsort of the buffer)
     + the level generator for the reset slots; ``new = active.at[ids].set(True)`` kept.
  2. ``_compute_algorithmic_regret`` (:293-329) per agent: a fresh A2C antagonist trained for
     ``max_lifetime`` updates (toued.a2c), then eval(A2C) - eval(LPG) over ``env_workers`` workers.
  3. the terminated agents' scores / flags scattered into the buffer (:188-200).
  4. toued_plr_sample: replay ids (rank or proportional), random new ids, the bernoulli/permutation
     selection (:203-227); ``active[new_ids] = True`` (:232-234).

Multi-GPU: the buffer is replicated on every rank and updated identically; each rank scores
its own agents and the per-agent (term, score, buffer id) vectors are all-gathered, so every
rank runs the same single-workgroup sampler kernel on the same inputs.

Scores of agents that are not terminated are discarded by the reference (``term_mask_fn``);
by default they are not computed (``regret_all_agents=False``): the regret of agent i depends
only on its own key, level and actor, so skipping the masked-out ones changes no output.
"""
from __future__ import annotations

import os

import torch

from . import _lib, prng
from .a2c import A2CHyperparams, A2CTrainer
from .debug import nan_checker
from .agents import AgentBatch, create_agents, eval_agent, eval_agent_reset
from .env import L_BUFID


def _split2(rng):
    if rng.dim() == 2:                 # a batch of keys: both halves contiguous from one planar split
        ks = prng.split_planar(rng, 2)
        return ks[0], ks[1]
    ks = prng.split(rng, 2)
    return ks[..., 0, :].contiguous(), ks[..., 1, :].contiguous()


def reset_lowest_scoring(sampler, rng: torch.Tensor, buffer, n_new: int) -> torch.Tensor:
    """level_sampler.py:331-353, in place on ``buffer``; returns the reset ids [n_new]."""
    B = len(buffer)
    ids = torch.empty(n_new, dtype=torch.int32, device=buffer.score.device)
    _lib.call("toued_plr_reset_ids", B, n_new, _lib.ptr(buffer.score), _lib.ptr(buffer.active),
              _lib.ptr(buffer.new), _lib.ptr(ids), _lib.stream_ptr())
    keys = prng.split(rng, n_new)
    levels = sampler.gen(keys, buffer_ids=ids)
    il = ids.long()
    buffer.levels.index_copy_(0, il, levels)
    buffer.score.index_fill_(0, il, 0.0)
    new = buffer.active.clone()
    new.index_fill_(0, il, True)
    buffer.active.index_fill_(0, il, False)
    buffer.new = new
    return ids


def algorithmic_regret(sampler, keys: torch.Tensor, levels: torch.Tensor, lpg_theta: torch.Tensor) -> torch.Tensor:
    """_compute_algorithmic_regret (level_sampler.py:293-329) for n agents (keys [n,2])."""
    n = keys.shape[0]
    if n == 0:
        return torch.zeros(0, device=keys.device)
    ro = sampler.rollout_manager
    W = sampler.env_workers
    rng, c = _split2(keys)
    w_rng, ag_rng = _split2(c)                       # _create_agent (:273-291)
    (_, _), state = ro.batch_reset(w_rng, levels, W)
    theta, vcrit = create_agents(ag_rng, ro.obs_dim, 1)   # value critic: critic_dims=1 (:280-281)
    vcrit = vcrit.reshape(n, ro.obs_dim).contiguous()
    rng, tr = _split2(rng)
    step = torch.zeros(n, dtype=torch.int32, device=keys.device)
    lpg_rng, a2c_rng = _split2(rng)
    # both eval_agent calls as one batch of 2n agents (each agent's rollout depends only on its own key, level and
    # table: bit-identical to two calls, at about the latency of one -- the returns-only rollout is latency-bound).
    # eval_agent's keys, reset and draws do not depend on the tables: the draws are made beside the antagonist's
    # update chain, and after it only the env chain runs (eval_agent_reset / eval_returns_from_draws, bit-identical)
    ev_levels = torch.cat([levels, levels])
    ev_state, ev_keys = eval_agent_reset(ro, torch.cat([lpg_rng, a2c_rng]), ev_levels, W)
    split_eval = (os.environ.get("TOUED_REGRET_SPLIT_EVAL", "1") != "0"
                  and _eval_draw_bytes(ro, 2 * n, W) <= EVAL_DRAWS_MAX_BYTES)
    trainer = sampler.a2c_trainer()
    trainer.train(tr, theta, vcrit, step, levels, state, sampler.max_lifetime,
                  eval_keys=ev_keys if split_eval else None, eval_levels=ev_levels if split_eval else None)
    both = torch.cat([lpg_theta, theta])
    if split_eval:
        cum = ro.eval_returns_from_draws(trainer.eval_draws_out, both, ev_levels, ev_state)
    else:
        cum = ro.eval_returns(ev_keys, both, ev_levels, ev_state)
    r = cum.mean(dim=1)
    r_lpg, r_a2c = r[:n], r[n:]
    return r_a2c - r_lpg


# the regret round's eval draws ([eval_len][2n * W][4] u32, plus as much key-chain scratch) are made ahead when they fit
EVAL_DRAWS_MAX_BYTES = 4 << 30


def _eval_draw_bytes(ro, n_agents: int, W: int) -> int:
    return 2 * 16 * ro.eval_rollout_len * n_agents * W


def _scatter_into(dst: torch.Tensor, ids: torch.Tensor, val) -> None:
    """dst[ids] = val for ids in [0, B], where id B (= len(dst)) is a sink whose writes are dropped."""
    ext = torch.empty(dst.shape[0] + 1, dtype=dst.dtype, device=dst.device)
    ext[:-1].copy_(dst)
    if isinstance(val, torch.Tensor):
        ext.index_put_((ids,), val.to(dst.dtype))
    else:   # a Python scalar goes in as a kernel argument (a host tensor would be copied in behind a stream sync)
        ext.index_fill_(0, ids, val)
    dst.copy_(ext[:-1])


def plr_sample(sampler, rng: torch.Tensor, buffer, agents: AgentBatch, term: torch.Tensor, sl=None):
    """Returns (rng, buffer, new_levels [n_local, 64]) — new_levels for terminated agents, the
    caller keeps the old level elsewhere (``term_mask_fn``)."""
    world = sampler.world
    N = agents.n if sl is None else sl[2]
    B = len(buffer)
    dev = agents.levels.device
    rng, sub = _split2(rng)
    # _reset_lowest_scoring touches only the buffer, which the regret round below does not read: it runs on a side
    # stream beside the antagonists' training, joined before the buffer update
    main = torch.cuda.current_stream()
    side = getattr(sampler, "_plr_side", None)
    if side is None:
        side = sampler._plr_side = torch.cuda.Stream(device=dev)
    side.wait_stream(main)
    # the side kernels read `sub` and the old `buffer.new` (both from main's allocator pool) after this function has
    # dropped them: keep their blocks from being reused by main until the side stream's work has passed them
    sub.record_stream(side)
    buffer.new.record_stream(side)
    with torch.cuda.stream(side):
        reset_lowest_scoring(sampler, sub, buffer, N)
    rng, sub = _split2(rng)
    keys = prng.split(sub, N)
    if sl is not None:
        keys = keys[sl[0]:sl[1]].contiguous()
    score = torch.zeros(agents.n, dtype=torch.float32, device=dev)
    if sampler.regret_all_agents:
        score = algorithmic_regret(sampler, keys, agents.levels, agents.theta)
    else:
        sel = term.nonzero().flatten()
        if sel.numel():
            score[sel] = algorithmic_regret(sampler, keys[sel].contiguous(), agents.levels[sel].contiguous(),
                                            agents.theta[sel].contiguous())
    nan_checker().check("regret_scores", score)
    old_ids = agents.levels[:, L_BUFID].contiguous()
    if world is not None and world.active:
        term_g = world.all_gather_cat(term.to(torch.int32)).bool()
        score_g = world.all_gather_cat(score)
        old_g = world.all_gather_cat(old_ids)
    else:
        term_g, score_g, old_g = term, score, old_ids
    main.wait_stream(side)
    buffer.new.record_stream(main)     # allocated on the side stream
    # buffer update for terminated levels (:188-200), without a boolean-mask gather (a host sync that would hold the
    # host's launches of the rest of sample() until the regret round has finished): every agent scatters, the
    # non-terminated ones into a sink slot B past the buffer's end
    t_ids = torch.where(term_g, old_g.long(), B)
    _scatter_into(buffer.score, t_ids, score_g)
    _scatter_into(buffer.active, t_ids, False)
    _scatter_into(buffer.new, t_ids, False)
    # replay vs random (:203-227)
    ks = prng.split(rng, 3)                           # rng, replay_rng, random_rng
    kbuf = torch.stack([ks[1], ks[2], ks[0]]).contiguous()
    chosen = torch.empty(N, dtype=torch.int32, device=dev)
    rep, rnd, use = torch.empty_like(chosen), torch.empty_like(chosen), torch.empty_like(chosen)
    _lib.call("toued_plr_sample", B, N, _lib.ptr(buffer.score), _lib.ptr(buffer.active), _lib.ptr(buffer.new),
              _lib.ptr(kbuf), int(sampler.score_transform == "proportional"), float(sampler.score_temperature),
              float(sampler.p_replay), _lib.ptr(chosen), _lib.ptr(rep), _lib.ptr(rnd), _lib.ptr(use),
              _lib.stream_ptr())
    sampler.last_plr = {"replay": rep, "random": rnd, "use": use, "chosen": chosen, "score": score_g}
    r1, _ = _split2(ks[0].contiguous())               # bernoulli: rng, _rng = split(rng)
    rng, _ = _split2(r1)                              # permutation: rng, _rng = split(rng)
    new_ids = torch.where(term_g, chosen, old_g)
    buffer.active.index_fill_(0, new_ids.long(), True)   # (:232-234)
    lo, hi = (0, N) if sl is None else (sl[0], sl[1])
    new_levels = buffer.levels[new_ids[lo:hi].long()]
    return rng, buffer, new_levels
