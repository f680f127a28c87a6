"""Checkpoint container (toued/checkpoint.py): flax 0.6.11 msgpack encoding restated (parity unpinned: flax
and no reference checkpoint are available), round trips of the LPG TrainState state dict and the level buffer,
and the save/restore file protocol of flax.training.checkpoints (legacy path)."""
import os

import msgpack
import numpy as np
import torch


def test_ndarray_leaf_encoding():
    from toued.checkpoint import msgpack_serialize
    a = np.arange(6, dtype=np.float32).reshape(2, 3)
    raw = msgpack.unpackb(msgpack_serialize({"a": a, "s": np.int32(7)}), raw=False)
    ext = raw["a"]
    assert isinstance(ext, msgpack.ExtType) and ext.code == 1
    shape, name, buf = msgpack.unpackb(ext.data, raw=False)
    assert shape == [2, 3] and name == "float32" and buf == a.tobytes("C")
    assert raw["s"].code == 3


def test_roundtrip_and_chunking(monkeypatch):
    from toued import checkpoint as ck
    monkeypatch.setattr(ck, "MAX_CHUNK_SIZE", 64)
    tree = {"x": np.random.RandomState(0).randn(7, 5).astype(np.float32), "n": {"i": np.arange(3, dtype=np.int32)},
            "e": {}, "c": 1 + 2j}
    raw = msgpack.unpackb(ck.msgpack_serialize(tree), raw=False, ext_hook=lambda c, d: msgpack.ExtType(c, d))
    assert raw["x"]["__msgpack_chunked_array__"] is True and len(raw["x"]["chunks"]) == 3
    back = ck.msgpack_restore(ck.msgpack_serialize(tree))
    assert np.array_equal(back["x"], tree["x"]) and np.array_equal(back["n"]["i"], tree["n"]["i"])
    assert back["e"] == {} and back["c"] == 1 + 2j


def test_lpg_train_state_roundtrip(tmp_path):
    from toued.checkpoint import lpg_flat_from_tree, lpg_train_state_dict, restore_checkpoint, save_checkpoint
    from toued.lpg import LPGLayout
    from toued.meta import AdamState
    for F in (5, 7):
        lay = LPGLayout(F)
        eta = torch.randn(lay.size)
        adam = AdamState(lay.size, "cpu")
        adam.m.normal_()
        adam.v.uniform_()
        adam.count = 12
        d = lpg_train_state_dict(eta, lay, 40, adam)
        g = d["params"]["LPGGRU_0"]["GRUCell_0"]
        assert g["hn"]["kernel"].shape == (256, 256) and g["in"]["kernel"].shape == (F, 256)
        assert set(g["hr"]) == {"kernel"} and d["params"]["MLP_0"]["Dense_1"]["kernel"].shape == (16, 1)
        assert sorted(d["opt_state"]) == ["0", "1", "2"] and d["opt_state"]["1"] == {}
        for step in (10, 40):
            save_checkpoint(str(tmp_path / f"F{F}"), d, step)
        assert sorted(os.listdir(tmp_path / f"F{F}")) == ["checkpoint_40"]   # keep=1
        r = restore_checkpoint(str(tmp_path / f"F{F}"))
        assert int(r["step"]) == 40 and int(r["opt_state"]["0"]["count"]) == 12
        assert np.array_equal(lpg_flat_from_tree(r["params"], lay), eta.numpy())
        assert np.array_equal(lpg_flat_from_tree(r["opt_state"]["0"]["mu"], lay), adam.m.numpy())
        assert np.array_equal(lpg_flat_from_tree(r["opt_state"]["0"]["nu"], lay), adam.v.numpy())


def test_level_buffer_reference_layout_roundtrip(tmp_path):
    """The buffer checkpoint is the reference's LevelBuffer pytree (level_sampler.py:30-52, util/data.py:46-51,
    gridworld.py:21-35): EnvParams fields in dataclass order with per-type object tables; packing it back gives
    the same device rows, for a tabular, an all_* and a mazes (manual dispatch, zero-padded types) buffer."""
    from oracle import jaxrand as jr
    from oracle import levels as olv
    from toued.checkpoint import (level_buffer_from_state_dict, level_buffer_state_dict, restore_checkpoint,
                                  save_checkpoint)
    from toued.env import get_env_spec
    from toued.level_sampler import LevelBuffer
    for mode in ("dense", "all_shortlife", "mazes", "tabular"):
        B = 40
        spec_o = olv.env_spec(mode)
        p, lt = olv.reset_env_params(jr.split(jr.PRNGKey(3), B), mode)
        packed = olv.pack_levels(p, lt, spec_o, np.arange(B, dtype=np.int32))
        rs = np.random.RandomState(1)
        buf = LevelBuffer(torch.from_numpy(packed), torch.from_numpy(rs.randn(B).astype(np.float32)),
                          torch.from_numpy(rs.rand(B) < 0.3), torch.from_numpy(rs.rand(B) < 0.5))
        spec, _, _ = get_env_spec(mode)
        d = level_buffer_state_dict(buf, spec)
        assert list(d) == ["level", "score", "active", "new"]
        assert list(d["level"]) == ["env_params", "lifetime", "buffer_id"]
        ep = d["level"]["env_params"]
        assert list(ep) == ["max_steps_in_episode", "random_respawn", "auto_collect", "grid_size", "walls",
                            "start_pos", "n_objs", "obj_ids", "static_obj_poss", "obj_rewards", "obj_p_terminate",
                            "obj_p_respawn"]
        for k in ("max_steps_in_episode", "grid_size", "start_pos", "n_objs", "obj_ids", "static_obj_poss", "walls"):
            assert np.array_equal(ep[k], p[k]), (mode, k)
        for k in ("obj_rewards", "obj_p_terminate", "obj_p_respawn"):
            assert np.array_equal(ep[k], p[k].astype(np.float32)), (mode, k)
        assert ep["auto_collect"].all() and np.array_equal(ep["random_respawn"], p["random_respawn"])
        assert np.array_equal(d["level"]["lifetime"], lt) and np.array_equal(d["level"]["buffer_id"], np.arange(B))
        save_checkpoint(str(tmp_path / mode), d, 3, prefix="buffer_")
        back = level_buffer_from_state_dict(restore_checkpoint(str(tmp_path / mode), prefix="buffer_"), spec, "cpu")
        assert torch.equal(back.levels, buf.levels) and torch.equal(back.score, buf.score)
        assert torch.equal(back.active, buf.active) and torch.equal(back.new, buf.new)


def test_es_train_state_layout():
    """ESTrainState (util/data.py:63-68) with evosax 0.1.4 OpenES EvoParams / EvoState field order (restated)."""
    from toued.checkpoint import es_train_state_dict, msgpack_restore, msgpack_serialize
    from toued.es import OpenES
    from toued.lpg import LPGLayout
    lay = LPGLayout(7)
    es = OpenES(8, lay.size, "adam", 0.01, 0.999, 1e-5, 0.1, 0.999, 0.01, 0.0, "cpu")
    es.mean.normal_()
    d = es_train_state_dict(es, torch.randn(lay.size), lay, "adam")
    assert list(d) == ["train_state", "es_params", "es_state"]
    assert list(d["es_state"]) == ["mean", "sigma", "opt_state", "best_member", "best_fitness", "gen_counter"]
    assert list(d["es_state"]["opt_state"]) == ["lrate", "m", "v", "n", "last_grads", "gen_counter"]
    assert list(d["es_params"]) == ["opt_params", "sigma_init", "sigma_decay", "sigma_limit", "init_min", "init_max",
                                    "clip_min", "clip_max"]
    assert float(d["es_params"]["opt_params"]["beta_1"]) == np.float32(0.99)
    r = msgpack_restore(msgpack_serialize(d))
    assert np.array_equal(r["es_state"]["mean"], es.mean.numpy()) and r["es_state"]["opt_state"]["n"] is None
    assert r["train_state"]["params"]["LPGGRU_0"]["GRUCell_0"]["in"]["kernel"].shape == (7, 256)
