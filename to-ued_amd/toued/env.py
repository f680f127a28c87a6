"""GridWorld on MI355X: level generation and the gymnax env API over the C ABI.

Mirrors environments/gridworld/gridworld.py (GridWorld: reset/step),
environments/environments.py:22-63 (get_env / reset_env_params / get_env_spec /
get_agent_hypers) and configs.py's mode tables — batched ("vmapped") over
levels/workers, with all state resident on the GPU.

Levels are packed int32[n, 80] tensors (include/toued.h); env state is
int32[12, n] SoA; observations are compact (tab_idx, time) int32 pairs.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _lib
from . import modes as M

STATE_FIELDS = 12
LEVEL_WORDS = 80
# packed-level word offsets (csrc/common.h)
L_MAX_STEPS, L_GRID, L_START, L_NOBJS, L_RANDRESP, L_LIFETIME, L_BUFID = 0, 1, 2, 3, 4, 5, 6
L_OBJ_IDS, L_STATIC, L_REW, L_PTERM, L_PRESP, L_WALLS = 8, 16, 24, 32, 40, 48
L_TREW, L_TPTERM, L_TPRESP, L_AUTOC = 64, 69, 74, 79


def unpack_levels(levels, spec: "EnvSpec"):
    """Packed rows [B, 80] -> the reference's Level pytree fields (util/data.py:46-51; EnvParams
    gridworld.py:21-35) as numpy arrays: ({EnvParams field: array}, lifetime, buffer_id)."""
    import numpy as np
    lv = np.ascontiguousarray(levels.detach().cpu().numpy() if torch.is_tensor(levels) else levels, np.int32)
    n, t, g2 = spec.max_n_objs, spec.max_n_obj_types, spec.g2
    bits = lv[:, L_WALLS:L_WALLS + 8].view(np.uint32)
    cells = np.arange(g2)
    walls = ((bits[:, cells // 32] >> (cells % 32).astype(np.uint32)) & 1).astype(bool)
    f = lambda off: lv[:, off:off + t].view(np.float32).copy()
    params = {
        "max_steps_in_episode": lv[:, L_MAX_STEPS].copy(), "random_respawn": lv[:, L_RANDRESP].astype(bool),
        "auto_collect": lv[:, L_AUTOC].astype(bool), "grid_size": lv[:, L_GRID].copy(), "walls": walls,
        "start_pos": lv[:, L_START].copy(), "n_objs": lv[:, L_NOBJS].copy(),
        "obj_ids": lv[:, L_OBJ_IDS:L_OBJ_IDS + n].copy(), "static_obj_poss": lv[:, L_STATIC:L_STATIC + n].copy(),
        "obj_rewards": f(L_TREW), "obj_p_terminate": f(L_TPTERM), "obj_p_respawn": f(L_TPRESP),
    }
    return params, lv[:, L_LIFETIME].copy(), lv[:, L_BUFID].copy()


def pack_levels(params: dict, lifetime, buffer_id, spec: "EnvSpec"):
    """Inverse of unpack_levels: the packed rows (with the per-object tables resolved through obj_ids, a -1 id
    taking the last type as jnp.take does, gridworld.py:87,115,122) as an int32 numpy array [B, 80]."""
    import numpy as np
    B = np.asarray(params["start_pos"]).shape[0]
    n, t = spec.max_n_objs, spec.max_n_obj_types
    out = np.zeros((B, LEVEL_WORDS), np.int32)
    out[:, L_MAX_STEPS] = params["max_steps_in_episode"]
    out[:, L_GRID] = params["grid_size"]
    out[:, L_START] = params["start_pos"]
    out[:, L_NOBJS] = params["n_objs"]
    out[:, L_RANDRESP] = np.asarray(params["random_respawn"]).astype(np.int32)
    out[:, L_LIFETIME] = lifetime
    out[:, L_BUFID] = buffer_id
    ids = np.asarray(params["obj_ids"], np.int32)
    out[:, L_OBJ_IDS:L_OBJ_IDS + n] = ids
    out[:, L_STATIC:L_STATIC + n] = params["static_obj_poss"]
    rid = np.where(ids < 0, ids + t, ids)
    for off, toff, name in ((L_REW, L_TREW, "obj_rewards"), (L_PTERM, L_TPTERM, "obj_p_terminate"),
                            (L_PRESP, L_TPRESP, "obj_p_respawn")):
        tab = np.asarray(params[name], np.float32)
        out[:, off:off + n] = np.take_along_axis(tab, rid, axis=1).view(np.int32)
        out[:, toff:toff + t] = tab.view(np.int32)
    walls = np.asarray(params["walls"], bool)
    for c in range(walls.shape[1]):
        out[:, L_WALLS + c // 32] |= (walls[:, c].astype(np.int64) << (c % 32)).astype(np.uint32).view(np.int32)
    out[:, L_AUTOC] = np.asarray(params.get("auto_collect", True)).astype(np.int32)
    return out


@dataclass(frozen=True)
class EnvSpec:
    """Static env kwargs (configs.py:430-544)."""
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

    @property
    def num_actions(self) -> int:
        return 5  # gridworld.py:218-222


def get_env_spec(env_mode: str):
    """environments.py:40-55: (env spec, max_rollout_len, max_lifetime)."""
    if env_mode not in M.ENV_MODE_KWARGS:
        raise ValueError(f"Environment mode {env_mode} has no get env spec method.")
    k = M.ENV_MODE_KWARGS[env_mode]
    spec = EnvSpec(k["max_grid_size"], k["max_n_objs"], k["max_n_obj_types"], k["tabular"])
    return spec, M.ENV_MODE_EPISODE_LEN[env_mode], M.ENV_MODE_LIFETIME_MAX[env_mode]


def get_agent_hypers(env_mode: str) -> dict:
    """environments.py:58-63 / configs.py:652-707."""
    if env_mode not in M.MODE_AGENT_HYPERS:
        raise ValueError(f"Environment mode {env_mode} has no get agent hyperparameters method.")
    return dict(M.MODE_AGENT_HYPERS[env_mode])


def _dev(device=None):
    return torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())


class LevelGenerator:
    """Device ``reset_env_params`` (environments.py:22-37) for one env mode."""

    def __init__(self, env_mode: str, device=None):
        if env_mode not in M.ENV_MODE_PARAMS:
            raise ValueError(f"Environment mode {env_mode} not registered.")
        self.env_mode = env_mode
        self.spec, _, _ = get_env_spec(env_mode)
        prog = M.mode_program(env_mode)
        nbytes = int(_lib.lib().toued_mode_program_bytes())
        if prog.nbytes != nbytes:
            raise _lib.ToUEDError(f"ModeProgram size mismatch: host {prog.nbytes} vs device {nbytes}")
        self.program = torch.from_numpy(prog).to(_dev(device))

    def __call__(self, keys: torch.Tensor, buffer_ids: torch.Tensor | None = None, with_sub_mode=False):
        """keys int32[n,2] (threefry) -> levels int32[n, LEVEL_WORDS = 80] (lifetime and buffer_id packed in)."""
        n = keys.shape[0]
        levels = torch.empty((n, LEVEL_WORDS), dtype=torch.int32, device=keys.device)
        sub = torch.empty((n,), dtype=torch.int32, device=keys.device) if with_sub_mode else None
        if buffer_ids is not None:
            buffer_ids = buffer_ids.to(torch.int32).contiguous()
        _lib.call("toued_level_gen", _lib.ptr(self.program), _lib.ptr(keys.contiguous()), _lib.ptr(buffer_ids),
                  _lib.ptr(levels), _lib.ptr(sub), n, _lib.stream_ptr())
        return (levels, sub) if with_sub_mode else levels

    def regenerate(self, keys: torch.Tensor, levels: torch.Tensor, mask: torch.Tensor):
        """``levels[i] = self(keys)[i]`` in place for the i with ``mask[i]`` (u8) set (buffer_id 0)."""
        _lib.call("toued_level_gen_masked", _lib.ptr(self.program), _lib.ptr(keys.contiguous()), None,
                  _lib.ptr(levels), keys.shape[0], _lib.ptr(mask), _lib.stream_ptr())
        return levels


class GridWorld:
    """gymnax ``Environment`` API for GridWorld (gridworld.py:38-236), vectorised.

    ``reset(keys, levels, W)`` and ``step(keys, state, actions, levels, W)``
    apply to n = keys.shape[0] workers; worker i uses level ``i // W``.
    ``step`` includes gymnax's auto-reset (select(done, reset, stepped)).
    """

    def __init__(self, spec: EnvSpec):
        self.spec = spec
        self._c = _lib.env_spec_c(spec)

    @property
    def num_actions(self) -> int:
        return 5

    def reset(self, keys, levels, W: int = 1):
        n = keys.shape[0]
        dev = keys.device
        state = torch.zeros((STATE_FIELDS, n), dtype=torch.int32, device=dev)
        idx = torch.empty(n, dtype=torch.int32, device=dev)
        tm = torch.empty(n, dtype=torch.int32, device=dev)
        _lib.call("toued_gw_reset", self._c, _lib.ptr(levels), W, _lib.ptr(keys), _lib.ptr(state), _lib.ptr(idx),
                  _lib.ptr(tm), n, _lib.stream_ptr())
        return (idx, tm), state

    def step(self, keys, state, actions, levels, W: int = 1):
        n = keys.shape[0]
        dev = keys.device
        state = state.clone()
        idx = torch.empty(n, dtype=torch.int32, device=dev)
        tm = torch.empty(n, dtype=torch.int32, device=dev)
        rew = torch.empty(n, dtype=torch.float32, device=dev)
        done = torch.empty(n, dtype=torch.uint8, device=dev)
        _lib.call("toued_gw_step", self._c, _lib.ptr(levels), W, _lib.ptr(keys), _lib.ptr(state),
                  _lib.ptr(actions.to(torch.int32).contiguous()), _lib.ptr(idx), _lib.ptr(tm), _lib.ptr(rew),
                  _lib.ptr(done), n, _lib.stream_ptr())
        return (idx, tm), state, rew, done.bool()

    def obs_dense(self, idx, tm):
        """Materialise the reference's dense observation (gridworld.py:184-199) — debugging only."""
        D = self.spec.obs_dim
        out = torch.zeros((idx.shape[0], D), dtype=torch.float32, device=idx.device)
        out[torch.arange(idx.shape[0], device=idx.device), idx.long()] = 1.0
        out[:, -1] = tm.float() * torch.tensor(0.001, dtype=torch.float32)
        return out
