"""numpy restatement of the PLR level-buffer logic — test oracle.

environments/level_sampler.py:
  _reset_lowest_scoring  :331-353  (incl. SURVEY B.4: new = active.at[ids].set(True))
  sample (alg_regret)    :169-234  buffer update for terminated agents, replay vs random
  _replay_from_buffer    :355-390  (rank: flip(argsort(p))[:N]; proportional: Gumbel top-k)
  _sample_random_from_buffer :392-408 (Gumbel top-k over new & ~active)

Float reductions whose order XLA leaves open (the softmax-score sum over the
buffer) are fixed here as a sequential sum; the device kernel uses the same order.
"""
from __future__ import annotations

import numpy as np

from . import jaxrand as jr
from . import pmath

F32 = np.float32


def argsort_stable(x):
    return np.argsort(x, kind="stable")


def reset_lowest_scoring(score, active, new, N):
    """Returns (reset_ids [N], score', active', new')."""
    s = np.where(new, F32(-np.inf), score).astype(F32)
    s = np.where(active, F32(np.inf), s).astype(F32)
    ids = argsort_stable(s)[:N].astype(np.int32)
    score2 = score.copy()
    score2[ids] = 0.0
    active2 = active.copy()
    active2[ids] = False
    new2 = active.copy()          # B.4: `new = active.at[ids].set(True)`
    new2[ids] = True
    return ids, score2, active2, new2


def seq_sum(x):
    s = F32(0.0)
    for v in x.astype(F32):
        s = F32(s + v)
    return s


def replay_ids(key, score, active, new, N, transform="rank", temperature=1.0):
    invalid = new | active
    sc = pmath.exp((score / F32(temperature)).astype(F32))
    sc = np.where(invalid, F32(0.0), sc).astype(F32)
    sc = (sc / seq_sum(sc)).astype(F32)
    B = score.shape[0]
    p = np.ones_like(sc) if (B - int(invalid.sum())) < N else sc
    if transform == "rank":
        return argsort_stable(p)[::-1][:N].astype(np.int32)
    ks = jr.split(key, 2)
    return jr.choice_p_noreplace(ks[1], p, N)


def random_ids(key, active, new, N):
    mask = new & ~active
    p = np.where(mask, F32(1.0), F32(0.0)).astype(F32)
    p = (p / seq_sum(p)).astype(F32)
    return jr.choice_p_noreplace(key, p, N)


def select(key, rep_ids, rnd_ids, active, new, N, p_replay):
    """level_sampler.py:211-229 (before the terminated mask): chosen buffer ids per agent."""
    ks = jr.split(key, 2)
    rng, sub = ks[0], ks[1]
    n_rep = int(np.sum(jr.uniform(sub, (N,)) < F32(p_replay)))
    use = np.arange(N) < n_rep
    n_replayable = len(active) - int(np.sum(new | active))
    use = use & (n_replayable >= N)
    ks = jr.split(rng, 2)
    use = jr.permutation(ks[1], use.astype(np.int32)).astype(bool)
    return np.where(use, rep_ids, rnd_ids).astype(np.int32), use
