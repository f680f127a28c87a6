"""Hand-derived known answers for the oracle GridWorld (gridworld.py:72-211)."""
import numpy as np

from oracle import gridworld as gw
from oracle import jaxrand as jr
from oracle import levels as lv

SPEC = gw.EnvSpec(max_grid_size=5, max_n_objs=2, max_n_obj_types=2, tabular=True)


def _params(B=1, walls=(), grid=4, start=0, objs=(6, 9), ids=(0, 1), rew=(1.0, -1.0), pterm=(0.0, 1.0),
            presp=(0.0, 0.0), max_steps=10, n_objs=2):
    w = np.zeros((B, 25), bool)
    for c in walls:
        w[:, c] = True
    rep = lambda v, dt: np.broadcast_to(np.asarray(v, dt), (B,) + np.shape(v)).copy()
    return {"max_steps_in_episode": rep(max_steps, np.int32), "random_respawn": rep(False, bool),
            "grid_size": rep(grid, np.int32), "walls": w, "start_pos": rep(start, np.int32),
            "n_objs": rep(n_objs, np.int32), "obj_ids": rep(ids, np.int32), "static_obj_poss": rep(objs, np.int32),
            "obj_rewards": rep(rew, np.float32), "obj_p_terminate": rep(pterm, np.float32),
            "obj_p_respawn": rep(presp, np.float32)}


def _state(pos, time=0, exists=(True, True), objs=(6, 9), ids=(0, 1), early=False):
    return {"time": np.array([time], np.int32), "pos": np.array([pos], np.int32),
            "obj_poss": np.array([[o + i * 25 for o, i in zip(objs, ids)]], np.int32),
            "obj_existss": np.array([exists]), "early_term": np.array([early])}


def test_border_clamp_and_walls():
    p = _params(walls=(5,))
    for pos, a, exp in [(0, 0, 0), (0, 2, 0), (3, 3, 3), (15, 1, 15), (0, 1, 4), (1, 1, 1),
                        (5, 4, 5), (6, 2, 6), (2, 3, 3), (2, 1, 6)]:
        got = gw.next_pos(np.array([pos]), np.array([a]), p)[0]
        assert got == exp, (pos, a, got, exp)


def test_collect_reward_and_termination():
    p = _params(pterm=(0.0, 1.0))
    # move right from 5 -> 6 collects object 0 (reward +1, p_term 0)
    s, r, d = gw.step_env(SPEC, jr.PRNGKey(0)[None], _state(5), np.array([3]), p)
    assert r[0] == 1.0 and not d[0] and not s["obj_existss"][0, 0] and s["obj_existss"][0, 1]
    assert s["pos"][0] == 6 and s["time"][0] == 1
    # move down from 5 -> 9 collects object 1 (reward -1, p_term 1 -> terminates)
    s, r, d = gw.step_env(SPEC, jr.PRNGKey(0)[None], _state(5), np.array([1]), p)
    assert r[0] == -1.0 and d[0] and s["early_term"][0]


def test_respawn_certain_and_unused_masked():
    p = _params(presp=(1.0, 1.0), n_objs=1)
    s, r, d = gw.step_env(SPEC, jr.PRNGKey(1)[None], _state(0, exists=(False, False)), np.array([4]), p)
    # object 0 respawns (p=1); object 1 is unused (n_objs=1) and stays masked
    assert s["obj_existss"][0].tolist() == [True, False]


def test_time_limit_done_and_auto_reset():
    p = _params(max_steps=3)
    st, r, d = gw.env_step(SPEC, jr.PRNGKey(2)[None], _state(0, time=2), np.array([4]), p)
    assert d[0] and st["time"][0] == 0 and st["pos"][0] == 0 and st["obj_existss"][0].all()


def test_tabular_index_formula():
    st = _state(7, exists=(False, True))
    idx, tm = gw.obs_compact(SPEC, st)
    assert idx[0] == 7 + 25 * 2
    dense = gw.obs_dense(SPEC, {**st, "time": np.array([12], np.int32)})
    assert dense.shape[1] == 25 * 4 + 1 and dense[0, 57] == 1.0 and dense[0].sum() == 1.0 + np.float32(12 * 0.001)


def test_isin_bool_walls_quirk():
    spec = gw.EnvSpec(5, 2, 2, False)
    p = _params(walls=(12,))
    v = gw.valid_obj_idxs(spec, np.array([3]), p)[0]
    # walls is a bool array containing both values -> cells 0 and 1 excluded; the wall cell 12 is NOT excluded
    assert not v[0] and not v[1] and v[12] and not v[3] and not v[16]
    p2 = _params(walls=())
    v2 = gw.valid_obj_idxs(spec, np.array([3]), p2)[0]
    assert not v2[0] and v2[1]


def test_take_wraps_negative_obj_ids():
    tab = np.array([[0.1, 0.2, 0.3]], np.float32)
    assert gw._take_wrap(tab, np.array([[-1, 0]]), 3).tolist() == [[np.float32(0.3), np.float32(0.1)]]


def test_level_generator_properties():
    for mode in ("dense", "all_shortlife", "tabular", "mazes", "all_vrandlife", "small"):
        spec = lv.env_spec(mode)
        keys = jr.split(jr.PRNGKey(0), 64)
        p, lt = lv.reset_env_params(keys, mode)
        g = p["grid_size"]
        assert (p["start_pos"] < g * g).all()
        assert not p["walls"][np.arange(64), p["start_pos"]].any()
        cells = np.concatenate([p["start_pos"][:, None], p["static_obj_poss"]], 1)
        nvalid = (np.arange(spec.g2)[None] < (g * g)[:, None]) & ~p["walls"]
        for b in range(64):
            used = cells[b, :1 + spec.max_n_objs]
            real = used[used >= 0]
            if nvalid[b].sum() >= len(real):
                assert len(set(real[: 1 + p["n_objs"][b]].tolist())) == 1 + p["n_objs"][b]
        assert (lt > 0).all()
