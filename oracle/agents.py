"""numpy restatement of agent creation and evaluation — test oracle.

agents/agents.py:31-56  create_agent: actor_rng, critic_rng = split(rng); each TrainState's
                        params = model.init(rng, ones(obs_shape)) (models/agent.py:7-45)
flax 0.6.11 (setup/requirements-base.txt:4, not vendored) initialises the Dense kernel with
  key = fold_in(rng, sha1("Dense_0" + b"\x01")[:4] big-endian)   (core/scope.py lazy RNG: the module
        path and the 'params' counter hashed together, oracle/flaxinit.py)
  lecun_normal = truncated_normal(key, -2, 2, (D, cols)) * sqrt(1/D) / .87962566103423978
agents/agents.py:98-106 eval_agent.
This derivation is restated from the flax sources' published algorithm; no reference output
pins it (parity unpinned beyond the PRNG known-answer vectors).
"""
from __future__ import annotations

import numpy as np

from . import flaxinit
from . import jaxrand as jr
from . import rollout as oro


def lecun_table(key, D: int, cols: int) -> np.ndarray:
    return flaxinit.dense0_table(key, D, cols)


def create_agent(key, D: int, critic_dims: int):
    ks = jr.split(key, 2)
    return lecun_table(ks[0], D, 5), lecun_table(ks[1], D, critic_dims)


def eval_agent(spec, keys, params, theta, W: int, L: int):
    """Per-agent mean first-episode return over W workers: keys [N,2], theta [N,D,5], params
    for the N agents (oracle/levels.py layout).  The mean is taken in float64."""
    ks = jr.split(keys, 2)
    st = oro.batch_reset(spec, ks[:, 1], params, W)
    ks2 = jr.split(ks[:, 0], 2)
    _, _, cum = oro.batch_rollout(spec, ks2[:, 1], theta, params, st, L)
    return cum.astype(np.float64).mean(axis=1)
