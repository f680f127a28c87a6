"""numpy restatement of RolloutWrapper + the linear-softmax tabular actor — test oracle.

Follows environments/rollout.py:38-102 (batch_reset / batch_rollout /
single_rollout.policy_step) and models/agent.py:7-17 (Actor with
``actor_net=()``: ``softmax(obs @ W)``, no bias; configs.py:652-659).

Observations are kept in the compact form (tab_idx, time): the reference's
dense one-hot obs dotted with W equals ``W[tab_idx] + (f32(time)*0.001)*W[D-1]``
(the zero terms contribute nothing).  This oracle fixes that sum as two
separately rounded f32 operations; ``obs_dense @ W`` agrees within 1 ulp.

Batched over agents: keys [N,2], level params with leading N, actor tables
theta[N, D, A]; workers W per agent.
"""
from __future__ import annotations

import numpy as np

from . import gridworld as gw
from . import jaxrand as jr
from . import pmath

F32 = np.float32
TIME_SCALE = F32(0.001)


def gather_rows(table, idx):
    """table [N, D, K], idx [N, ...] -> [N, ..., K]."""
    N = table.shape[0]
    lead = idx.shape
    flat_idx = idx.reshape(N, -1)
    out = table[np.arange(N)[:, None], flat_idx]
    return out.reshape(lead + (table.shape[-1],))


def logits_of(table, idx, time):
    """table [N, D, K]; idx/time [N, ...] -> f32 logits [N, ..., K]."""
    N, D, K = table.shape
    c = (time.astype(F32) * TIME_SCALE)[..., None]
    rows = gather_rows(table, idx)
    last = table[:, D - 1, :].reshape((N,) + (1,) * (idx.ndim - 1) + (K,))
    return (rows + c * last).astype(F32)


def softmax(logits):
    """jax.nn.softmax with the portable exp and a sequential sum."""
    m = np.max(logits, axis=-1, keepdims=True)
    e = pmath.exp(logits - m)
    s = e[..., 0]
    for j in range(1, e.shape[-1]):
        s = s + e[..., j]
    return (e / s[..., None]).astype(F32)


def _tile_params(params, W):
    return {k: np.repeat(v, W, axis=0) for k, v in params.items()}


def batch_reset(spec, keys, params, W):
    """rollout.py:38-42 for N agents: split(rng, W) then vmap(env.reset)."""
    N = keys.shape[0]
    wk = jr.split(keys, W).reshape(N * W, 2)
    tp = _tile_params(params, W)
    state = gw.env_reset(spec, wk, tp)
    return state


def batch_rollout(spec, keys, theta, params, state, T):
    """rollout.py:45-102.  Returns (traj, end_state, cum_return[N,W]).

    traj: idx/time int32[N,W,T+1] (obs_t for t<T, end obs at T; next_obs_t == obs_{t+1}),
          action int32[N,W,T], reward f32[N,W,T], done bool[N,W,T].
    """
    N = keys.shape[0]
    W = state["pos"].shape[0] // N
    rng = jr.split(keys, W).reshape(N * W, 2)
    tp = _tile_params(params, W)
    idx_l, time_l, act_l, rew_l, done_l = [], [], [], [], []
    cum = np.zeros(N * W, F32)
    valid = np.ones(N * W, F32)
    for t in range(T):
        ks = jr.split(rng, 2)
        rng, sub = ks[:, 0], ks[:, 1]
        idx, tm = gw.obs_compact(spec, state)
        probs = softmax(logits_of(theta, idx.reshape(N, W), tm.reshape(N, W))).reshape(N * W, -1)
        action = jr.choice_p_replace(sub, probs)
        ks = jr.split(rng, 2)
        rng, sub = ks[:, 0], ks[:, 1]
        state, reward, done = gw.env_step(spec, sub, state, action, tp)
        cum = cum + reward * valid
        valid = valid * (F32(1.0) - done.astype(F32))
        idx_l.append(idx)
        time_l.append(tm)
        act_l.append(action)
        rew_l.append(reward)
        done_l.append(done)
    idx, tm = gw.obs_compact(spec, state)
    idx_l.append(idx)
    time_l.append(tm)
    sh = lambda a: np.stack(a, axis=1).reshape((N, W) + np.stack(a, axis=1).shape[1:])
    traj = {"idx": sh(idx_l), "time": sh(time_l), "action": sh(act_l), "reward": sh(rew_l), "done": sh(done_l)}
    return traj, state, cum.reshape(N, W)
