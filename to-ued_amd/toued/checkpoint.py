"""Checkpoints of the LPG train state and the level buffer (experiments/logging.py:31-46 of the reference).

The reference writes, after training, ``flax.training.checkpoints.save_checkpoint(ckpt_dir, target, step,
keep=1[, prefix="buffer_"])``: with flax 0.6.11's legacy (non-Orbax) path that is one file
``<ckpt_dir>/<prefix><step>`` (prefix "checkpoint_" by default) holding
``flax.serialization.msgpack_serialize(to_state_dict(target))``.

flax is not installed here, so its msgpack encoding is restated from flax/serialization.py (0.6.11) — parity
unpinned, no reference checkpoint exists to read back:
  * the state dict is packed with ``msgpack.packb(tree, default=ext_pack, strict_types=True)``;
  * ndarray leaves become ``ExtType(1, packb((shape, dtype.name, C-order bytes), use_bin_type=True))``, numpy
    scalars ``ExtType(3, ...)`` of the same payload for a 0-d array, complex numbers ``ExtType(2, packb((re, im)))``;
  * leaves over 2^30 bytes are replaced by ``{"__msgpack_chunked_array__": True, "shape": {"0": ...},
    "chunks": {"0": flat chunk, ...}}``.

``lpg_train_state_dict`` builds ``to_state_dict`` of the meta-gradient TrainState (meta/meta.py:10-30): ``step``,
``params`` (the flax module tree of models/lpg.py, see toued/lpg.py for the names) and ``opt_state`` of
``optax.chain(scale_by_adam(), scale(lr), scale(-1))`` = ``{"0": {"count", "mu", "nu"}, "1": {}, "2": {}}``
(apply_fn and tx are static fields and not serialised).

``level_buffer_state_dict`` writes the reference's ``LevelBuffer`` pytree (level_sampler.py:30-52): ``level``
= ``Level(env_params, lifetime, buffer_id)`` (util/data.py:46-51) with every ``EnvParams`` field
(gridworld.py:21-35, per-type object tables included: the packed rows carry them), then ``score``, ``active``,
``new`` -- in dataclass field order, as flax's to_state_dict emits them.  ``es_train_state_dict`` writes
``ESTrainState`` (util/data.py:63-68): ``train_state`` (the LPG TrainState, which the ES step never updates),
``es_params`` and ``es_state`` of evosax 0.1.4's OpenES (EvoParams / EvoState with the optimiser's
OptParams / OptState; evosax is not installed or vendored: field names, order and defaults restated, unpinned).
"""
from __future__ import annotations

import enum
import os
from collections import OrderedDict

import msgpack
import numpy as np
import torch

MAX_CHUNK_SIZE = 2 ** 30

# flat LPG layout name -> path in the flax params tree (models/lpg.py: Dense_0 = pi head, Dense_1 = y head,
# LPGGRU_0/GRUCell_0 = the reverse GRU, MLP_0 = the embedding net)
_PARAM_PATHS = OrderedDict([
    ("pi_b", ("Dense_0", "bias")), ("pi_w", ("Dense_0", "kernel")),
    ("y_b", ("Dense_1", "bias")), ("y_w", ("Dense_1", "kernel")),
    ("hn_b", ("LPGGRU_0", "GRUCell_0", "hn", "bias")), ("hn_w", ("LPGGRU_0", "GRUCell_0", "hn", "kernel")),
    ("hr_w", ("LPGGRU_0", "GRUCell_0", "hr", "kernel")), ("hz_w", ("LPGGRU_0", "GRUCell_0", "hz", "kernel")),
    ("in_b", ("LPGGRU_0", "GRUCell_0", "in", "bias")), ("in_w", ("LPGGRU_0", "GRUCell_0", "in", "kernel")),
    ("ir_b", ("LPGGRU_0", "GRUCell_0", "ir", "bias")), ("ir_w", ("LPGGRU_0", "GRUCell_0", "ir", "kernel")),
    ("iz_b", ("LPGGRU_0", "GRUCell_0", "iz", "bias")), ("iz_w", ("LPGGRU_0", "GRUCell_0", "iz", "kernel")),
    ("e1_b", ("MLP_0", "Dense_0", "bias")), ("e1_w", ("MLP_0", "Dense_0", "kernel")),
    ("e2_b", ("MLP_0", "Dense_1", "bias")), ("e2_w", ("MLP_0", "Dense_1", "kernel")),
])


class _Ext(enum.IntEnum):
    ndarray = 1
    native_complex = 2
    npscalar = 3


def _ndarray_to_bytes(arr: np.ndarray) -> bytes:
    if arr.dtype.hasobject or arr.dtype.isalignedstruct:
        raise ValueError("object and structured dtypes cannot be serialised")
    return msgpack.packb((arr.shape, arr.dtype.name, arr.tobytes("C")), use_bin_type=True)


def _ndarray_from_bytes(data: bytes) -> np.ndarray:
    shape, dtype_name, buf = msgpack.unpackb(data, raw=True)
    return np.frombuffer(buf, dtype=np.dtype(dtype_name.decode()), count=-1, offset=0).reshape(shape, order="C")


def _ext_pack(x):
    if isinstance(x, np.ndarray):
        return msgpack.ExtType(_Ext.ndarray, _ndarray_to_bytes(x))
    if isinstance(x, np.generic):
        return msgpack.ExtType(_Ext.npscalar, _ndarray_to_bytes(np.asarray(x)))
    if isinstance(x, complex):
        return msgpack.ExtType(_Ext.native_complex, msgpack.packb((x.real, x.imag)))
    return x


def _ext_unpack(code, data):
    if code == _Ext.ndarray:
        return _ndarray_from_bytes(data)
    if code == _Ext.native_complex:
        re, im = msgpack.unpackb(data)
        return complex(re, im)
    if code == _Ext.npscalar:
        return _ndarray_from_bytes(data)[()]
    return msgpack.ExtType(code, data)


def _to_numpy(tree):
    if isinstance(tree, dict):
        return {str(k): _to_numpy(v) for k, v in tree.items()}
    if isinstance(tree, torch.Tensor):
        return tree.detach().cpu().numpy()
    return tree


def _chunk(arr: np.ndarray) -> dict:
    size = max(1, int(MAX_CHUNK_SIZE / arr.dtype.itemsize))
    flat = arr.reshape(-1)
    chunks = [flat[i:i + size] for i in range(0, flat.size, size)]
    return {"__msgpack_chunked_array__": True, "shape": {str(i): s for i, s in enumerate(arr.shape)},
            "chunks": {str(i): c for i, c in enumerate(chunks)}}


def _chunk_leaves(tree):
    if isinstance(tree, dict):
        return {k: (_chunk(v) if isinstance(v, np.ndarray) and v.size * v.dtype.itemsize > MAX_CHUNK_SIZE
                    else _chunk_leaves(v)) for k, v in tree.items()}
    return tree


def _unchunk_leaves(tree):
    if isinstance(tree, dict):
        if tree.get("__msgpack_chunked_array__") is True:
            shape = tuple(tree["shape"][str(i)] for i in range(len(tree["shape"])))
            flat = np.concatenate([tree["chunks"][str(i)] for i in range(len(tree["chunks"]))])
            return flat.reshape(shape)
        return {k: _unchunk_leaves(v) for k, v in tree.items()}
    return tree


def msgpack_serialize(tree) -> bytes:
    """flax.serialization.msgpack_serialize of a state dict (dicts with str keys; ndarray / tensor / scalar leaves)."""
    return msgpack.packb(_chunk_leaves(_to_numpy(tree)), default=_ext_pack, strict_types=True)


def msgpack_restore(data: bytes):
    """flax.serialization.msgpack_restore: the state dict back, ndarray leaves as read-only numpy views."""
    return _unchunk_leaves(msgpack.unpackb(data, ext_hook=_ext_unpack, raw=False))


def _nest(flat: dict) -> dict:
    out: dict = {}
    for path, v in flat.items():
        d = out
        for key in path[:-1]:
            d = d.setdefault(key, {})
        d[path[-1]] = v
    return out


def lpg_params_tree(eta: torch.Tensor, lay) -> dict:
    """The flax params tree of the flat LPG vector (toued/lpg.py layout)."""
    e = eta.detach().cpu().numpy().astype(np.float32)
    return _nest({_PARAM_PATHS[k]: e[lay.offsets[k]:lay.offsets[k] + int(np.prod(s))].reshape(s).copy()
                  for k, s in lay.shapes.items()})


def lpg_flat_from_tree(params: dict, lay) -> np.ndarray:
    """Inverse of lpg_params_tree (checks every leaf's shape)."""
    out = np.zeros(lay.size, np.float32)
    for k, s in lay.shapes.items():
        v = params
        for key in _PARAM_PATHS[k]:
            v = v[key]
        v = np.asarray(v, np.float32)
        if v.shape != tuple(s):
            raise ValueError(f"checkpoint leaf {'/'.join(_PARAM_PATHS[k])}: shape {v.shape} != {tuple(s)}")
        out[lay.offsets[k]:lay.offsets[k] + v.size] = v.reshape(-1)
    return out


def lpg_train_state_dict(eta: torch.Tensor, lay, step: int, adam=None) -> dict:
    """to_state_dict(TrainState) of the meta-gradient LPG (meta/meta.py:24) with its Adam chain state."""
    count = 0 if adam is None else int(adam.count)
    zeros = torch.zeros_like(eta)
    return {"step": np.asarray(step, np.int32),
            "params": lpg_params_tree(eta, lay),
            "opt_state": {"0": {"count": np.asarray(count, np.int32),
                                "mu": lpg_params_tree(zeros if adam is None else adam.m, lay),
                                "nu": lpg_params_tree(zeros if adam is None else adam.v, lay)},
                          "1": {}, "2": {}}}


def level_buffer_state_dict(buffer, spec) -> dict:
    """to_state_dict(LevelBuffer) of the reference (level_sampler.py:30-52) from the packed device buffer."""
    from .env import unpack_levels
    params, lifetime, buffer_id = unpack_levels(buffer.levels, spec)
    return {"level": {"env_params": params, "lifetime": lifetime.astype(np.int32), "buffer_id": buffer_id.astype(np.int32)},
            "score": buffer.score.detach().cpu().numpy().astype(np.float32),
            "active": buffer.active.detach().cpu().numpy().astype(bool),
            "new": buffer.new.detach().cpu().numpy().astype(bool)}


def level_buffer_from_state_dict(state: dict, spec, device):
    """A reference (or this build's) buffer checkpoint back into the device LevelBuffer."""
    from .env import pack_levels
    from .level_sampler import LevelBuffer
    lv = state["level"]
    packed = pack_levels(lv["env_params"], np.asarray(lv["lifetime"]).astype(np.int32),
                         np.asarray(lv["buffer_id"]).astype(np.int32), spec)
    t = lambda a, dt: torch.as_tensor(np.array(a), dtype=dt, device=device)
    return LevelBuffer(t(packed, torch.int32), t(state["score"], torch.float32), t(state["active"], torch.bool),
                       t(state["new"], torch.bool))


_F32_MAX = float(np.finfo(np.float32).max)


def es_train_state_dict(es, eta_train_state: torch.Tensor, lay, lpg_opt: str, best_member=None,
                        best_fitness=_F32_MAX) -> dict:
    """to_state_dict(ESTrainState) (util/data.py:63-68; meta/meta.py:24-30).  ``es`` is toued.es.OpenES;
    ``eta_train_state`` the params of the wrapped TrainState (the LPG init: lpg_es_train_step only replaces
    es_state, meta/train.py:214-216).  evosax 0.1.4 OpenES: EvoParams(opt_params, sigma_init, sigma_decay,
    sigma_limit, init_min=0, init_max=0, clip_min=-f32max, clip_max=f32max), EvoState(mean, sigma, opt_state,
    best_member, best_fitness, gen_counter); Adam/SGD OptParams(lrate_init, lrate_decay, lrate_limit, momentum,
    beta_1, beta_2, beta_3, eps, max_speed) and OptState(lrate, m, v, n, last_grads, gen_counter)."""
    f = lambda x: np.asarray(x, np.float32)
    adam = es.opt == 1
    nd = es.nd
    opt_params = {"lrate_init": f(es.lrate_init), "lrate_decay": f(es.lrate_decay), "lrate_limit": f(es.lrate_limit),
                  "momentum": None if adam else f(0.0), "beta_1": f(0.99) if adam else None,
                  "beta_2": f(0.999) if adam else None, "beta_3": None, "eps": f(1e-8) if adam else None,
                  "max_speed": None}
    es_params = {"opt_params": opt_params, "sigma_init": f(es.sigma_init), "sigma_decay": f(es.sigma_decay),
                 "sigma_limit": f(es.sigma_limit), "init_min": f(0.0), "init_max": f(0.0), "clip_min": f(-_F32_MAX),
                 "clip_max": f(_F32_MAX)}
    mean = es.mean.detach().cpu().numpy().astype(np.float32)
    opt_state = {"lrate": f(es.lrate), "m": es.m.detach().cpu().numpy().astype(np.float32),
                 "v": es.v.detach().cpu().numpy().astype(np.float32) if adam else None, "n": None, "last_grads": None,
                 "gen_counter": np.asarray(es.n, np.int32)}
    bm = mean if best_member is None else (best_member.detach().cpu().numpy() if torch.is_tensor(best_member)
                                           else np.asarray(best_member)).astype(np.float32)
    es_state = {"mean": mean, "sigma": f(es.sigma), "opt_state": opt_state, "best_member": bm,
                "best_fitness": f(best_fitness), "gen_counter": np.asarray(es.gen_counter, np.int32)}
    if lpg_opt.lower() == "adam":
        zeros = torch.zeros(lay.size)
        tx_state = {"0": {"count": np.asarray(0, np.int32), "mu": lpg_params_tree(zeros, lay),
                          "nu": lpg_params_tree(zeros, lay)}, "1": {}, "2": {}}
    else:   # optax.chain(clip_by_global_norm, scale, scale): three empty states
        tx_state = {"0": {}, "1": {}, "2": {}}
    train_state = {"step": np.asarray(0, np.int32), "params": lpg_params_tree(eta_train_state, lay),
                   "opt_state": tx_state}
    return {"train_state": train_state, "es_params": es_params, "es_state": es_state}


def save_checkpoint(ckpt_dir: str, target: dict, step: int, prefix: str = "checkpoint_", keep: int = 1) -> str:
    """flax.training.checkpoints.save_checkpoint (legacy msgpack path): write ``<prefix><step>`` through a
    temporary file, then keep only the ``keep`` newest ``<prefix>*`` checkpoints."""
    os.makedirs(ckpt_dir, exist_ok=True)
    path = os.path.join(ckpt_dir, f"{prefix}{step}")
    tmp = os.path.join(ckpt_dir, f"{prefix}tmp")
    with open(tmp, "wb") as f:
        f.write(msgpack_serialize(target))
    os.replace(tmp, path)
    olds = sorted((p for p in os.listdir(ckpt_dir) if p.startswith(prefix) and p[len(prefix):].isdigit()),
                  key=lambda p: int(p[len(prefix):]))
    for p in olds[:-keep] if keep > 0 else []:
        os.remove(os.path.join(ckpt_dir, p))
    return path


def restore_checkpoint(ckpt_dir: str, prefix: str = "checkpoint_", step: int | None = None):
    """flax.training.checkpoints.restore_checkpoint(target=None): the newest (or the given) step's state dict."""
    if step is None:
        steps = [int(p[len(prefix):]) for p in os.listdir(ckpt_dir) if p.startswith(prefix) and p[len(prefix):].isdigit()]
        if not steps:
            raise FileNotFoundError(f"no {prefix}* checkpoint in {ckpt_dir}")
        step = max(steps)
    with open(os.path.join(ckpt_dir, f"{prefix}{step}"), "rb") as f:
        return msgpack_restore(f.read())
