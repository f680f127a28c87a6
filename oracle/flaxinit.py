"""flax 0.6.11 parameter initialisation restated in numpy — test oracle (test infrastructure only).

The reference initialises every network with ``model.init(rng, ...)``:
  * LPG:    meta/meta.py:21-22  ``lpg_model.init(rng, *lpg_model.get_init_vector())["params"]``
            (models/lpg.py:38-96: MLP_0 embedding, LPGGRU_0/GRUCell_0 under nn.scan with
            split_rngs={"params": False}, the Dense_0 / Dense_1 heads)
  * agents: agents/agents.py:78-80 ``model.init(rng, jnp.ones(obs_shape))`` of Actor / Critic
            (models/agent.py:7-45 with actor_net=(): one ``nn.Dense(n, use_bias=False)`` = Dense_0)

flax 0.6.11 (setup/requirements-base.txt:4) is not installed and not vendored; this restates its
published algorithm (flax/core/scope.py, flax/linen/recurrent.py, jax/_src/nn/initializers.py):

  param key   Scope.make_rng("params") = LazyRng(root, suffix).as_jax_rng() with the lazy-RNG default
              (config flax_lazy_rng = True): suffix = the module path names, then the scope's 'params'
              counter (1 for the first param of a module = its kernel); _fold_in_static hashes the whole
              suffix at once — sha1 over the utf-8 names and the counter's minimal big-endian bytes, no
              separator (flax_fix_rng_separator = False) — and folds the first 4 digest bytes (big-endian
              uint32) into the root key with ONE jax.random.fold_in.
  nn.scan     split_rngs={"params": False} broadcasts the scope's LazyRng unchanged into the scanned body,
              so the GRU kernels see suffix [LPGGRU_0, GRUCell_0, <gate>, 1].
  Dense       kernel_init lecun_normal = variance_scaling(1, "fan_in", "truncated_normal"):
              truncated_normal(key, -2, 2, shape) * (sqrt(f32(1/fan_in)) / f32(.87962566103423978)),
              fan_in = shape[-2]; bias zeros.
  GRUCell     input kernels ir/iz/in: lecun_normal (Dense with bias, zeros); recurrent hr/hz: orthogonal(),
              no bias; hn: orthogonal() with a zero bias.
  orthogonal  A = normal(key, (n, n)); Q, R = qr(A); Q *= sign(diag(R)).  jnp.linalg.qr runs LAPACK in f32;
              here the QR is float64 of the same f32 A, rounded once (differences ~1e-7, below the 1e-6 the
              tests allow between implementations; the random draws themselves are bit-exact).

Parity unpinned beyond the PRNG known answers: no flax output is available offline.
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict

import numpy as np

from . import jaxrand as jr
from .lpg import layout

F32 = np.float32
TN_STD_DIV = F32(0.87962566103423978)


def static_hash(path) -> int:
    """flax core/scope.py _fold_in_static: sha1 over the suffix elements, first 4 bytes big-endian."""
    m = hashlib.sha1()
    for x in path:
        if isinstance(x, str):
            m.update(x.encode("utf-8"))
        elif isinstance(x, int):
            m.update(x.to_bytes((x.bit_length() + 7) // 8, byteorder="big"))
        else:
            raise ValueError(x)
    return int.from_bytes(m.digest()[:4], "big")


def param_key(rng, path) -> np.ndarray:
    """The key ``self.param(...)`` receives for the parameter at module path + counter ``path``."""
    if len(path) == 0:
        return np.asarray(rng, np.uint32)
    return jr.fold_in(rng, static_hash(path))


def lecun_std(fan_in: int) -> np.float32:
    return F32(np.sqrt(F32(1.0 / fan_in))) / TN_STD_DIV


def lecun_normal(key, shape) -> np.ndarray:
    return (jr.truncated_normal(key, -2.0, 2.0, shape) * lecun_std(shape[-2])).astype(F32)


def orthogonal(key, n: int) -> np.ndarray:
    a = jr.normal(key, (n, n)).astype(np.float64)
    q, r = np.linalg.qr(a)
    return (q * np.sign(np.diag(r))[None, :]).astype(F32)


GRU = ("LPGGRU_0", "GRUCell_0")
# layout name -> (init, module path); biases are zeros
LPG_PARAM_PATHS = {
    "pi_w": ("lecun", ("Dense_0",)),
    "y_w": ("lecun", ("Dense_1",)),
    "hn_w": ("orth", GRU + ("hn",)),
    "hr_w": ("orth", GRU + ("hr",)),
    "hz_w": ("orth", GRU + ("hz",)),
    "in_w": ("lecun", GRU + ("in",)),
    "ir_w": ("lecun", GRU + ("ir",)),
    "iz_w": ("lecun", GRU + ("iz",)),
    "e1_w": ("lecun", ("MLP_0", "Dense_0")),
    "e2_w": ("lecun", ("MLP_0", "Dense_1")),
}


def lpg_init(rng, F: int) -> np.ndarray:
    """create_lpg_train_state's params (meta/meta.py:21-22) as the flat f32 vector in jax tree order
    (oracle/lpg.py layout)."""
    parts = OrderedDict()
    for name, shape in layout(F).items():
        if name.endswith("_b"):
            parts[name] = np.zeros(shape, F32)
            continue
        kind, path = LPG_PARAM_PATHS[name]
        key = param_key(rng, path + (1,))
        parts[name] = orthogonal(key, shape[0]) if kind == "orth" else lecun_normal(key, shape)
    return np.concatenate([p.ravel() for p in parts.values()]).astype(F32)


def dense0_table(rng, D: int, cols: int) -> np.ndarray:
    """Actor / Critic with actor_net=() (models/agent.py:7-45): the Dense_0 kernel [D, cols]."""
    return lecun_normal(param_key(rng, ("Dense_0", 1)), (D, cols))
