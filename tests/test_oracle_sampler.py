"""CPU checks of the PLR buffer / A2C oracles (oracle/sampler.py, oracle/a2c.py, oracle/agents.py).

The reference has no tests or fixtures for this path; these pin the
restatement against the semantics of level_sampler.py:331-408 on hand-made cases and
check the A2C oracle's gradient against finite differences.
"""
import numpy as np
import torch

from oracle import a2c as oa2c
from oracle import agents as oag
from oracle import jaxrand as jr
from oracle import meta as ometa
from oracle import sampler as osp

F32 = np.float32


def test_reset_prefers_new_then_lowest_and_skips_active():
    score = np.array([0.5, -1.0, 2.0, 0.0, -0.0, 3.0], F32)
    active = np.array([0, 1, 0, 0, 0, 0], bool)
    new = np.array([0, 0, 0, 0, 0, 1], bool)
    ids, s2, a2, n2 = osp.reset_lowest_scoring(score, active, new, 4)
    # new (-inf) first, then scores ascending with -0 == 0 ties by index, active (inf) last
    assert ids.tolist() == [5, 3, 4, 0]
    assert s2[ids].tolist() == [0.0] * 4
    assert not a2[ids].any()
    # new := active.at[ids].set(True) — level 1 (active) stays flagged new
    assert n2.tolist() == [True, True, False, True, True, True]


def test_rank_replay_orders_by_score_ties_descending_index():
    score = np.array([1.0, 3.0, 3.0, -2.0, 0.0, 5.0], F32)
    active = np.zeros(6, bool)
    new = np.zeros(6, bool)
    new[5] = True
    ids = osp.replay_ids(jr.PRNGKey(0), score, active, new, 4, "rank")
    # level 5 invalid (p = 0); equal p for 1 and 2 -> flip(stable argsort) lists 2 before 1
    assert ids.tolist() == [2, 1, 0, 4]


def test_replay_uniform_when_too_few_valid():
    score = np.arange(8, dtype=F32)
    active = np.zeros(8, bool)
    new = np.ones(8, bool)
    new[:2] = False
    ids = osp.replay_ids(jr.PRNGKey(0), score, active, new, 4, "rank")
    assert ids.tolist() == [7, 6, 5, 4]    # p = ones -> flip(arange)


def test_random_ids_draw_only_new_inactive():
    B, N = 200, 30
    rs = np.random.RandomState(0)
    active = rs.rand(B) < 0.2
    new = (rs.rand(B) < 0.5) & ~active
    for s in range(5):
        ids = osp.random_ids(jr.PRNGKey(s), active, new, N)
        assert len(set(ids.tolist())) == N
        assert (new[ids] & ~active[ids]).all()


def test_proportional_replay_prefers_high_scores():
    B, N = 400, 50
    score = np.linspace(-3, 3, B).astype(F32)
    active = np.zeros(B, bool)
    new = np.zeros(B, bool)
    hits = np.zeros(B)
    for s in range(20):
        ids = osp.replay_ids(jr.PRNGKey(s), score, active, new, N, "proportional")
        assert len(set(ids.tolist())) == N
        hits[ids] += 1
    assert hits[B // 2:].sum() > 4 * hits[:B // 2].sum()


def test_select_counts_and_guard():
    B, N = 100, 16
    active = np.zeros(B, bool)
    new = np.zeros(B, bool)
    rep = np.arange(N, dtype=np.int32)
    rnd = np.arange(N, dtype=np.int32) + 50
    ch, use = osp.select(jr.PRNGKey(3), rep, rnd, active, new, N, 0.5)
    ks = jr.split(jr.PRNGKey(3), 2)
    assert use.sum() == int(np.sum(jr.uniform(ks[1], (N,)) < F32(0.5)))
    assert np.array_equal(ch, np.where(use, rep, rnd))
    new[:90] = True   # only 10 replayable < N -> never replay
    ch, use = osp.select(jr.PRNGKey(3), rep, rnd, active, new, N, 0.5)
    assert not use.any() and np.array_equal(ch, rnd)


def test_lecun_table_statistics():
    D = 3201
    t = oag.lecun_table(jr.PRNGKey(0), D, 5)
    std = np.sqrt(1.0 / D)
    assert t.dtype == np.float32 and t.shape == (D, 5)
    assert abs(t.std() / std - 1.0) < 0.03
    assert np.abs(t).max() <= 2.0 * std / 0.87962566103423978 + 1e-6


def _traj(W, T, D, seed):
    rs = np.random.RandomState(seed)
    return {"idx": rs.randint(0, D - 1, (W, T + 1)).astype(np.int32), "time": rs.randint(0, 50, (W, T + 1)).astype(np.int32),
            "action": rs.randint(0, 5, (W, T)).astype(np.int64), "reward": rs.randn(W, T).astype(np.float32),
            "done": rs.rand(W, T) < 0.1}


def test_a2c_oracle_update_matches_finite_differences():
    D, W, T = 40, 4, 6
    tr = _traj(W, T, D, 0)
    rs = np.random.RandomState(1)
    th = torch.from_numpy(rs.randn(D, 5)).double()
    vc = torch.from_numpy(rs.randn(D, 1)).double()
    hyp = ometa.Hypers()
    # with huge max_norm and lr = 1 the update is exactly -grad
    t1, v1, s1, al, cl = oa2c.a2c_step(th, vc, 0, 10, tr, hyp, 1.0, 1.0, 1e9)
    g = (th - t1).numpy()
    assert s1 == 1

    def actor_loss(theta):
        return oa2c.a2c_step(theta, vc, 0, 10, tr, hyp, 0.0, 0.0, 1e9)[3]
    eps = 1e-6
    for (i, j) in [(int(tr["idx"][0, 0]), int(tr["action"][0, 0])), (D - 1, 2), (int(tr["idx"][3, 4]), 0)]:
        tp, tm = th.clone(), th.clone()
        tp[i, j] += eps
        tm[i, j] -= eps
        fd = (actor_loss(tp) - actor_loss(tm)) / (2 * eps)
        assert abs(fd - g[i, j]) < 1e-6 * max(1.0, abs(fd)), (i, j, fd, g[i, j])
    # discard past the lifetime
    t2, v2, s2, _, _ = oa2c.a2c_step(th, vc, 10, 10, tr, hyp, 1.0, 1.0, 1e9)
    assert s2 == 10 and torch.equal(t2, th) and torch.equal(v2, vc)
