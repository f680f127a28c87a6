"""numpy restatement of OpenES as TO-UED configures it — test oracle.

models/optim.py:21-34 create_es_strategy -> evosax 0.1.4 OpenES (setup/requirements-base.txt:2,
not vendored, not installed: its published algorithm restated here; parity unpinned beyond the
PRNG known-answer vectors):
  initialize: mean = uniform(rng, (nd,), init_min=0, init_max=0) = 0; sigma = sigma_init;
              optimiser state m = v = 0, n = 0, lrate = lrate_init
  ask:        z = normal(rng, (P/2, nd)); x = mean + sigma * concat(z, -z); clip(-f32max, f32max)
  tell:       fitness' = -fitness (maximize); noise = (x - mean)/sigma;
              grad = 1/(P sigma) * noise^T fitness'; optimiser step; lrate = max(lrate*decay, limit);
              sigma = max(sigma*decay, limit)
  Adam:       m = (1-b1) g + b1 m; v = (1-b2) g^2 + b2 v; mhat = m/(1-b1^(n+1)); vhat = v/(1-b2^(n+1));
              mean -= lrate * mhat / (sqrt(vhat) + eps); b1 = .99, b2 = .999, eps = 1e-8 as float32 values (the
              OptParams leaves are traced as f32 arrays: 1 - b2 = 0.00099998713, not 0.001)
meta/train.py:152-158 reorders the population so candidates 2i and 2i+1 are z_i and -z_i;
meta/train.py:199-206 rank per antithetic pair.
"""
from __future__ import annotations

import numpy as np

from . import jaxrand as jr

F32 = np.float32


def ask(key, mean, sigma, popsize: int):
    nd = mean.shape[0]
    z = jr.normal(key, (popsize // 2, nd))
    x = np.concatenate([mean + F32(sigma) * z, mean + F32(sigma) * (F32(-1.0) * z)]).astype(F32)
    idxs = np.concatenate([[i, i + popsize // 2] for i in range(popsize // 2)])
    return x[idxs]


def pair_rank(fitness):
    fg = fitness[0::2] > fitness[1::2]
    rank = np.zeros_like(fitness, dtype=F32)
    rank[0::2] = fg.astype(F32)
    rank[1::2] = F32(1.0) - fg.astype(F32)
    return rank, fg


def tell(x, rank_fitness, state: dict, opt="adam"):
    """state: mean, sigma, m, v, n, lrate, lrate_decay, lrate_limit, sigma_decay, sigma_limit.
    Returns the new state (float64 accumulation of the population dot)."""
    return opt_step(grad(x, rank_fitness, state), state, opt)


def grad(x, rank_fitness, state):
    """the OpenES gradient 1/(P sigma) noise^T (-rank fitness) (maximize), float64"""
    P = x.shape[0]
    mean = state["mean"].astype(np.float64)
    sigma = float(state["sigma"])
    fit = -np.asarray(rank_fitness, np.float64)
    noise = (x.astype(np.float64) - mean) / sigma
    return (1.0 / (P * sigma)) * (noise.T @ fit)


def opt_step(g, state: dict, opt="adam"):
    """the optimiser step on the mean and the lrate / sigma decay, given the gradient g"""
    mean = state["mean"].astype(np.float64)
    s = dict(state)
    if opt == "adam":
        # evosax's OptParams (beta_1 .99, beta_2 .999, eps 1e-8) reach the jitted tell as float32 leaves
        b1, b2, eps = float(np.float32(0.99)), float(np.float32(0.999)), float(np.float32(1e-8))
        m = (1 - b1) * g + b1 * state["m"]
        v = (1 - b2) * g * g + b2 * state["v"]
        # the bias corrections as evosax's jitted f32 computes them: 1 - b2^(n+1) cancels (0.005 at n = 4), so its
        # float32 rounding (~1e-5 relative) shows in every update
        n1 = np.float32(state["n"] + 1)
        bc1 = float(np.float32(1.0) - np.float32(b1) ** n1)
        bc2 = float(np.float32(1.0) - np.float32(b2) ** n1)
        mhat = m / bc1
        vhat = v / bc2
        s["mean"] = mean - state["lrate"] * mhat / (np.sqrt(vhat) + eps)
        s["m"], s["v"] = m, v
    else:
        s["mean"] = mean - state["lrate"] * g
        s["m"] = g
    s["n"] = state["n"] + 1
    s["lrate"] = max(state["lrate"] * state["lrate_decay"], state["lrate_limit"])
    s["sigma"] = max(state["sigma"] * state["sigma_decay"], state["sigma_limit"])
    return s
