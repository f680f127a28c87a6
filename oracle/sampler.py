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


# ---------------------------------------------------------------------------
# LevelSampler.initial_sample / sample for the non-PLR score functions and the shared agent creation
# (level_sampler.py:90-167, 237-291).  Levels are (params dict, lifetime, buffer_id) triples with a leading
# batch axis; the caller packs them with oracle/levels.pack_levels.

def take_levels(lv, ids):
    p, lt, bid = lv
    return ({k: v[ids] for k, v in p.items()}, lt[ids], bid[ids])


def where_levels(mask, new, old):
    (pn, ln, bn), (po, lo, bo) = new, old
    sel = lambda a, b: np.where(mask.reshape((-1,) + (1,) * (a.ndim - 1)), a, b)
    return ({k: sel(pn[k], po[k]) for k in pn}, sel(ln, lo), sel(bn, bo))


def random_levels(key, mode, n):
    """_sample_random_levels (:268-271): split(rng, N) -> reset_env_params; buffer_id = 0 (float in the
    reference, B.10)."""
    from . import levels as olv
    p, lt = olv.reset_env_params(jr.split(key, n), mode)
    return p, lt, np.zeros(n, np.int32)


def initialize_buffer(key, mode, B):
    """initialize_buffer (:90-96): B levels from split(rng, B); score 0, active False, new True, id = i."""
    from . import levels as olv
    p, lt = olv.reset_env_params(jr.split(key, B), mode)
    return (p, lt, np.arange(B, dtype=np.int32)), np.zeros(B, F32), np.zeros(B, bool), np.ones(B, bool)


def create_agents(spec, keys, lv, W, Y):
    """vmap(_create_agent) (:273-291): worker_rng, agent_rng = split(rng_i); batch_reset(worker_rng, W);
    create_agent(agent_rng) -> (actor table [N,D,5], critic table [N,D,Y]), env state dict."""
    from . import agents as oag
    from . import rollout as oro
    ks = jr.split(keys, 2)
    st = oro.batch_reset(spec, ks[:, 0], lv[0], W)
    tabs = [oag.create_agent(ks[a, 1], spec.obs_dim, Y) for a in range(keys.shape[0])]
    return np.stack([t[0] for t in tabs]), np.stack([t[1] for t in tabs]), st


def value_critics(spec, key, n):
    """create_value_critic over split(rng, N) (:126-131, :249-255): lecun kernel [D, 1] per agent."""
    from . import agents as oag
    ks = jr.split(key, n)
    return np.stack([oag.lecun_table(ks[a], spec.obs_dim, 1) for a in range(n)])


def initial_sample(spec, mode, score_function, key, buffer_lv, n, W, Y, with_vc):
    """initial_sample (:103-132).  Only the random branch splits before the agents (:112-114)."""
    rng = key
    if score_function == "random":
        rng, sub = jr.split(rng, 2)
        lv = random_levels(sub, mode, n)
    else:
        lv = take_levels(buffer_lv, np.arange(n))
    rng, sub = jr.split(rng, 2)
    theta, phi, st = create_agents(spec, jr.split(sub, n), lv, W, Y)
    vc = None
    if with_vc:
        rng, sub = jr.split(rng, 2)
        vc = value_critics(spec, sub, n)
    return lv, theta, phi, st, vc


def sample_nonplr(spec, mode, score_function, key, buffer_lv, term, old, W, Y):
    """sample (:134-167, :237-266) for score_function random / frozen.  old = (levels, theta, phi, state,
    vcrit-or-None, step).  Returns the masked new (levels, theta, phi, state, vcrit, step)."""
    lv_old, th_old, ph_old, st_old, vc_old, step_old = old
    n = term.shape[0]
    rng = key
    if score_function == "random":
        rng, sub = jr.split(rng, 2)
        new_lv = random_levels(sub, mode, n)
    elif score_function == "frozen":
        B = buffer_lv[1].shape[0]
        p_uniform = np.full(B, F32(1.0) / F32(B), F32)      # jnp.ones((B,)) / B
        rng, sub = jr.split(rng, 2)
        ids = jr.choice_p_replace(sub, p_uniform, (n,))
        new_lv = take_levels(buffer_lv, ids)
    else:
        raise ValueError(score_function)
    lv = where_levels(term, new_lv, lv_old)
    rng, sub = jr.split(rng, 2)
    th, ph, st = create_agents(spec, jr.split(sub, n), lv, W, Y)
    t3 = term[:, None, None]
    th = np.where(t3, th, th_old)
    ph = np.where(t3, ph, ph_old)
    tw = np.repeat(term, W)
    st = {k: np.where(tw.reshape((-1,) + (1,) * (v.ndim - 1)), v, st_old[k]) for k, v in st.items()}
    vc = None
    if vc_old is not None:
        rng, sub = jr.split(rng, 2)
        vc = np.where(t3, value_critics(spec, sub, n), vc_old)
    step = np.where(term, 0, step_old)
    return lv, th, ph, st, vc, step
