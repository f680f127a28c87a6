"""numpy restatement of the GridWorld env + gymnax auto-reset wrapper — test oracle.

Follows environments/gridworld/gridworld.py:72-211 and gymnax 0.0.6
``Environment.step/reset`` (called at environments/rollout.py:41,65).
Batched over a leading axis B (one key/state/action per element); level
parameters are per-element arrays (leading axis B) as produced by
``oracle.levels``.

State dict (gridworld.py:11-18): time i32[B], pos i32[B], obj_poss i32[B,n],
obj_existss bool[B,n], early_term bool[B].  Params dict (gridworld.py:21-35):
max_steps_in_episode, random_respawn, grid_size, walls bool[B,G2], start_pos,
n_objs, obj_ids i32[B,n], static_obj_poss, obj_rewards/obj_p_terminate/
obj_p_respawn f32[B,n_types].
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import jaxrand as jr
from . import pmath

F32 = np.float32


@dataclass(frozen=True)
class EnvSpec:
    """Static env kwargs (configs.py:430-544 ENV_MODE_KWARGS)."""
    max_grid_size: int
    max_n_objs: int
    max_n_obj_types: int
    tabular: bool

    @property
    def g2(self) -> int:
        return self.max_grid_size ** 2

    @property
    def obs_dim(self) -> int:
        # gridworld.py:230-235
        if self.tabular:
            return self.g2 * (2 ** self.max_n_objs) + 1
        return self.g2 * (self.max_n_obj_types + 1) + 1


def _take_wrap(table, ids, n_types):
    """jnp.take(table, ids) with jax's default mode: negative ids wrap once (gridworld.py:87,115,122)."""
    idx = np.where(ids < 0, ids + n_types, ids)
    return np.take_along_axis(table, idx, axis=-1)


def next_pos(pos, action, params):
    """_get_next_pos, gridworld.py:138-146 (borders of the grid_size lattice, walls block)."""
    g = params["grid_size"]
    top = pos < g
    bottom = pos >= g * (g - 1)
    left = (pos % g) == 0
    right = (pos % g) == g - 1
    step = ((action == 0) * (1 - top) * -g + (action == 1) * (1 - bottom) * g
            + (action == 2) * (1 - left) * -1 + (action == 3) * (1 - right) * 1)
    nxt = (pos + step).astype(np.int32)
    wall = np.take_along_axis(params["walls"], nxt[:, None].astype(np.int64) % params["walls"].shape[1], axis=1)[:, 0]
    return np.where(wall, pos, nxt).astype(np.int32)


def valid_obj_idxs(spec: EnvSpec, pos, params):
    """_get_valid_obj_idxs, gridworld.py:149-155 — including the isin(idx, bool walls) quirk
    (SURVEY App. B.5): cells equal to a *value* of the bool walls array (0 and/or 1) are excluded,
    not the wall cells."""
    B = pos.shape[0]
    idx = np.broadcast_to(np.arange(spec.g2, dtype=np.int32), (B, spec.g2))
    walls = params["walls"]
    has_false = np.any(~walls, axis=1)
    has_true = np.any(walls, axis=1)
    in_walls = ((idx == 0) & has_false[:, None]) | ((idx == 1) & has_true[:, None])
    valid = (idx != pos[:, None]) & ~in_walls
    return valid & (idx < (params["grid_size"] ** 2)[:, None])


def tabular_pos(spec: EnvSpec, pos, exists):
    """_get_tabular_pos, gridworld.py:201-205."""
    pw = (2 ** np.arange(spec.max_n_objs)).astype(np.int32)
    return (pos + spec.g2 * np.sum(np.where(exists, pw, 0), axis=-1)).astype(np.int32)


def obs_compact(spec: EnvSpec, state):
    """Compact form of get_obs (gridworld.py:184-199) for the tabular env: the dense obs is the
    one-hot of ``tab_idx`` over D-1 cells followed by f32(time)*f32(0.001)."""
    return tabular_pos(spec, state["pos"], state["obj_existss"]), state["time"].astype(np.int32)


def obs_dense(spec: EnvSpec, state):
    """Dense get_obs (gridworld.py:184-199), float32[B, D]."""
    B = state["pos"].shape[0]
    obs = np.zeros((B, spec.obs_dim), dtype=F32)
    if spec.tabular:
        obs[np.arange(B), tabular_pos(spec, state["pos"], state["obj_existss"])] = 1.0
    else:
        obs[np.arange(B), state["pos"]] = 1.0
        for i in range(spec.max_n_objs):
            sel = state["obj_existss"][:, i]
            obs[np.arange(B)[sel], spec.g2 + state["obj_poss"][sel, i]] = 1.0
    obs[:, -1] = state["time"].astype(F32) * F32(0.001)
    return obs


def reset_env(spec: EnvSpec, key, params):
    """reset_env, gridworld.py:157-182."""
    B = key.shape[0]
    ks = jr.split(key, 2)
    obj_key = ks[:, 0]
    pos = params["start_pos"].astype(np.int32).copy()
    if spec.tabular:
        obj_poss = params["static_obj_poss"].astype(np.int32).copy()
    else:
        valid = valid_obj_idxs(spec, pos, params)
        p = (valid.astype(F32) / np.sum(valid, axis=1, keepdims=True).astype(F32)).astype(F32)
        rnd = jr.choice_p_noreplace(obj_key, p, spec.max_n_objs)
        obj_poss = np.where(params["random_respawn"][:, None], rnd, params["static_obj_poss"]).astype(np.int32)
    obj_poss = (obj_poss + params["obj_ids"] * spec.g2).astype(np.int32)
    exists = np.arange(spec.max_n_objs)[None, :] < params["n_objs"][:, None]
    return {
        "time": np.zeros(B, np.int32),
        "pos": pos,
        "obj_poss": obj_poss,
        "obj_existss": exists,
        "early_term": np.zeros(B, bool),
    }


def step_env(spec: EnvSpec, key, state, action, params):
    """step_env, gridworld.py:72-136.  Returns (state', reward f32[B], done bool[B])."""
    ks = jr.split(key, 3)
    term_key, respawn_key, obj_key = ks[:, 0], ks[:, 1], ks[:, 2]
    pos = next_pos(state["pos"], action, params)
    old = (state["obj_poss"] - params["obj_ids"] * spec.g2).astype(np.int32)
    collected = state["obj_existss"] & (old == pos[:, None])
    nt = spec.max_n_obj_types
    p_resp = _take_wrap(params["obj_p_respawn"], params["obj_ids"], nt)
    respawn = jr.uniform(respawn_key, (spec.max_n_objs,)) < p_resp
    exists = state["obj_existss"] | respawn
    if spec.tabular:
        obj_poss = old
    else:
        valid = valid_obj_idxs(spec, pos, params)
        for i in range(spec.max_n_objs):
            valid[np.arange(len(pos)), old[:, i]] = False
        p_vac = (valid.astype(F32) / np.sum(valid, axis=1, keepdims=True).astype(F32)).astype(F32)
        rnd = jr.choice_p_noreplace(obj_key, p_vac, spec.max_n_objs)
        use_new = (~state["obj_existss"]) & respawn
        new = np.where(use_new, rnd, old)
        obj_poss = np.where(params["random_respawn"][:, None], new, old)
    obj_poss = (obj_poss + params["obj_ids"] * spec.g2).astype(np.int32)
    exists = exists & ~collected
    exists = exists & (np.arange(spec.max_n_objs)[None, :] < params["n_objs"][:, None])
    p_term = _take_wrap(params["obj_p_terminate"], params["obj_ids"], nt)
    p_t = np.sum(p_term * collected.astype(F32), axis=1, dtype=F32)
    term = (jr.uniform(term_key, ()) < p_t) | state["early_term"]
    time = state["time"] + 1
    rew_t = _take_wrap(params["obj_rewards"], params["obj_ids"], nt)
    reward = np.sum(rew_t * collected.astype(F32), axis=1, dtype=F32) + F32(0.0)
    new_state = {"time": time.astype(np.int32), "pos": pos, "obj_poss": obj_poss,
                 "obj_existss": exists, "early_term": term}
    done = (time >= params["max_steps_in_episode"]) | term   # is_terminal, gridworld.py:207-211
    return new_state, reward.astype(F32), done


def env_step(spec: EnvSpec, key, state, action, params):
    """gymnax Environment.step: key,key_reset=split(key); step_env; reset_env; select(done)."""
    ks = jr.split(key, 2)
    key_s, key_r = ks[:, 0], ks[:, 1]
    st, reward, done = step_env(spec, key_s, state, action, params)
    re = reset_env(spec, key_r, params)
    out = {k: np.where(done.reshape((-1,) + (1,) * (st[k].ndim - 1)), re[k], st[k]) for k in st}
    return out, reward, done


def env_reset(spec: EnvSpec, key, params):
    """gymnax Environment.reset(key, params) = reset_env(key, params)."""
    return reset_env(spec, key, params)
