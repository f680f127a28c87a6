"""numpy restatement of the level generator — test oracle.

Follows environments/environments.py:22-37 (``reset_env_params``: split into
param/lifetime keys) and environments/gridworld/configs.py:12-126 (per-mode
parameter sampling, samplers ``uniform_first_pos/uniform_wall_idxs/log_uniform/
log_uniform_int``).  Vectorised over a batch of keys [B, 2].

Manual meta-modes (``tabular``, ``mazes``) crash in the reference
(configs.py:19-20 indexes ``mps["obj_ids"]`` on a manual entry -> KeyError;
SURVEY App. B.1).  This build DEFINES their dispatch (parity unpinned):
``sub_rng, rng = split(rng)``; ``i = randint(sub_rng, (), 0, len(modes))``;
the level is drawn from ``modes[i]`` with ``rng`` and zero/-1 padded to the
meta-mode's kwargs.
"""
from __future__ import annotations

import numpy as np

from . import jaxrand as jr
from . import pmath
from .gridworld import EnvSpec
from .modes import ENV_MODE_KWARGS, ENV_MODE_LIFETIME, ENV_MODE_PARAMS

F32 = np.float32


def env_spec(mode: str) -> EnvSpec:
    k = ENV_MODE_KWARGS[mode]
    return EnvSpec(k["max_grid_size"], k["max_n_objs"], k["max_n_obj_types"], k["tabular"])


def _log_bounds(lo, hi):
    """jnp.log(minval), jnp.log(maxval) evaluated in float32 (configs.py:119-120)."""
    return pmath.log(F32(lo)), pmath.log(F32(hi))


def sample_spec(key, spec, B):
    """Evaluate one distribution spec with a batch of keys [B,2] (the key is used directly)."""
    kind = spec[0]
    if kind == "const":
        v = np.asarray(spec[1])
        return np.broadcast_to(v, (B,) + v.shape).copy()
    if kind == "log_uniform_int":
        lo, hi = _log_bounds(spec[1], spec[2])
        u = jr.uniform(key, (), lo, hi)
        return np.rint(pmath.exp(u)).astype(np.int32)
    if kind == "log_uniform":
        lo, hi = _log_bounds(spec[2], spec[3])
        return pmath.exp(jr.uniform(key, (spec[1],), lo, hi))
    if kind == "uniform":
        return jr.uniform(key, (spec[1],), spec[2], spec[3])
    if kind == "uniform_first_pos":
        n, lo, hi = spec[1], spec[2], spec[3]
        ks = jr.split(key, 2)
        a = jr.uniform(ks[:, 0], (1,), 0.0, hi)
        b = jr.uniform(ks[:, 1], (n - 1,), lo, hi)
        return np.concatenate([a, b], axis=1)
    if kind == "choice_arange":
        lo, hi = spec[1], spec[2]
        return (lo + jr.randint(key, (), 0, hi - lo)).astype(np.int32)
    if kind == "wall_idxs":
        n_walls, mg = spec[1], spec[2]
        return jr.choice_noreplace(key, mg * mg, n_walls)
    raise ValueError(kind)


def _sample_obj_param(key, spec, n_types, B):
    """configs.py:75-80: callable -> sample then zero-pad; constant list -> zero-pad."""
    v = sample_spec(key, spec, B).astype(F32)
    pad = n_types - v.shape[1]
    return np.concatenate([v, np.zeros((B, pad), F32)], axis=1)


def _sample_param(key, spec, B):
    """configs.py:83-88: callables get an *extra* split (rng, _rng = split(rng); param(_rng))."""
    if spec[0] == "const":
        return sample_spec(key, spec, B)
    ks = jr.split(key, 2)
    return sample_spec(ks[:, 1], spec, B)


def reset_grid_params(key, mode: str):
    """configs.py:12-53 for a concrete mode; returns a params dict with leading batch B."""
    key = np.asarray(key, np.uint32)
    B = key.shape[0]
    mps = ENV_MODE_PARAMS[mode]
    kw = ENV_MODE_KWARGS[mode]
    n_max, n_types, mg = kw["max_n_objs"], kw["max_n_obj_types"], kw["max_grid_size"]
    p = {}
    p["obj_ids"] = np.broadcast_to(np.array(mps["obj_ids"] + [-1] * (n_max - len(mps["obj_ids"])), np.int32),
                                   (B, n_max)).copy()
    rng = key
    for name in ("obj_rewards", "obj_p_terminate", "obj_p_respawn"):
        ks = jr.split(rng, 2)
        rng, sub = ks[:, 0], ks[:, 1]
        p[name] = _sample_obj_param(sub, mps[name], n_types, B)
    p["random_respawn"] = np.full(B, not mps["tabular"])
    for name in ("max_steps_in_episode", "n_objs", "grid_size"):
        ks = jr.split(rng, 2)
        rng, sub = ks[:, 0], ks[:, 1]
        p[name] = _sample_param(sub, mps[name], B).astype(np.int32)
    ks = jr.split(rng, 2)
    rng, sub = ks[:, 0], ks[:, 1]
    wall_idxs = np.asarray(_sample_param(sub, mps["wall_idxs"], B)).astype(np.int32)
    if wall_idxs.ndim == 1:
        wall_idxs = wall_idxs[:, None]
    walls = np.zeros((B, mg * mg), bool)
    for i in range(wall_idxs.shape[1]):
        walls[np.arange(B), wall_idxs[:, i]] = True
    p["walls"] = walls
    all_pos = np.arange(mg * mg)
    valid = (all_pos[None, :] < (p["grid_size"] ** 2)[:, None]) & ~walls
    ks = jr.split(rng, 2)
    rng, sub = ks[:, 0], ks[:, 1]
    sampled = jr.choice_p_noreplace(sub, valid.astype(F32), n_max + 1)
    p["start_pos"] = sampled[:, 0].astype(np.int32)
    p["static_obj_poss"] = sampled[:, 1:].astype(np.int32)
    return p


def pad_params(p, src_kw, dst_kw):
    """Embed a sub-mode level into a manual meta-mode's (larger) static kwargs."""
    B = p["start_pos"].shape[0]
    n, t, g = dst_kw["max_n_objs"], dst_kw["max_n_obj_types"], dst_kw["max_grid_size"]
    q = dict(p)
    sn = p["obj_ids"].shape[1]
    q["obj_ids"] = np.concatenate([p["obj_ids"], np.full((B, n - sn), -1, np.int32)], 1)
    q["static_obj_poss"] = np.concatenate([p["static_obj_poss"], np.zeros((B, n - sn), np.int32)], 1)
    for name in ("obj_rewards", "obj_p_terminate", "obj_p_respawn"):
        st = p[name].shape[1]
        q[name] = np.concatenate([p[name], np.zeros((B, t - st), F32)], 1)
    sg2 = p["walls"].shape[1]
    q["walls"] = np.concatenate([p["walls"], np.zeros((B, g * g - sg2), bool)], 1)
    return q


def reset_env_params(key, mode: str):
    """environments.py:22-37: (params, lifetime) for a batch of keys [B,2]."""
    key = np.asarray(key, np.uint32)
    B = key.shape[0]
    ks = jr.split(key, 2)
    p_rng, l_rng = ks[:, 0], ks[:, 1]
    mps = ENV_MODE_PARAMS[mode]
    if mps.get("manual"):
        subs = mps["modes"]
        ks2 = jr.split(p_rng, 2)
        sub_rng, rng = ks2[:, 0], ks2[:, 1]
        choice = jr.randint(sub_rng, (), 0, len(subs))
        out = None
        for i, sm in enumerate(subs):
            sel = choice == i
            if not np.any(sel):
                continue
            pi = pad_params(reset_grid_params(rng[sel], sm), ENV_MODE_KWARGS[sm], ENV_MODE_KWARGS[mode])
            if out is None:
                out = {k: np.zeros((B,) + v.shape[1:], v.dtype) for k, v in pi.items()}
            for k, v in pi.items():
                out[k][sel] = v
        params = out
        params["sub_mode"] = choice.astype(np.int32)
    else:
        params = reset_grid_params(p_rng, mode)
        params["sub_mode"] = np.zeros(B, np.int32)
    lifetime = sample_spec(l_rng, ENV_MODE_LIFETIME[mode], B).astype(np.int32)
    return params, lifetime


# ---------------------------------------------------------------------------
# Packed device layout (int32[80] per level) shared with the HIP kernels.
LEVEL_WORDS = 80
L_MAX_STEPS, L_GRID, L_START, L_NOBJS, L_RANDRESP, L_LIFETIME, L_BUFID = 0, 1, 2, 3, 4, 5, 6
L_OBJ_IDS, L_STATIC, L_REW, L_PTERM, L_PRESP, L_WALLS = 8, 16, 24, 32, 40, 48
L_TREW, L_TPTERM, L_TPRESP, L_AUTOC = 64, 69, 74, 79    # per-type EnvParams tables, auto_collect


def pack_levels(params, lifetime, spec: EnvSpec, buffer_id=None) -> np.ndarray:
    """Pack params into int32[B, 80]: scalars, raw obj_ids, static positions, the per-object
    resolved type tables (jnp.take with -1 wrap, gridworld.py:87,115,122), a walls bitmask, and the
    per-type tables + auto_collect of EnvParams (gridworld.py:21-35) for the checkpoint round trip."""
    B = params["start_pos"].shape[0]
    n = spec.max_n_objs
    out = np.zeros((B, LEVEL_WORDS), np.int32)
    out[:, L_MAX_STEPS] = params["max_steps_in_episode"]
    out[:, L_GRID] = params["grid_size"]
    out[:, L_START] = params["start_pos"]
    out[:, L_NOBJS] = params["n_objs"]
    out[:, L_RANDRESP] = params["random_respawn"].astype(np.int32)
    out[:, L_LIFETIME] = lifetime
    out[:, L_BUFID] = 0 if buffer_id is None else buffer_id
    ids = params["obj_ids"].astype(np.int32)
    out[:, L_OBJ_IDS:L_OBJ_IDS + n] = ids
    out[:, L_STATIC:L_STATIC + n] = params["static_obj_poss"]
    rid = np.where(ids < 0, ids + spec.max_n_obj_types, ids)
    for off, name in ((L_REW, "obj_rewards"), (L_PTERM, "obj_p_terminate"), (L_PRESP, "obj_p_respawn")):
        tab = np.take_along_axis(params[name].astype(F32), rid, axis=1)
        out[:, off:off + n] = tab.view(np.int32)
    walls = params["walls"]
    for c in range(walls.shape[1]):
        w = c // 32
        out[:, L_WALLS + w] |= (walls[:, c].astype(np.int64) << (c % 32)).astype(np.uint32).view(np.int32)
    nt = params["obj_rewards"].shape[1]
    for off, name in ((L_TREW, "obj_rewards"), (L_TPTERM, "obj_p_terminate"), (L_TPRESP, "obj_p_respawn")):
        out[:, off:off + nt] = params[name].astype(F32).view(np.int32)
    out[:, L_AUTOC] = 1
    return out
