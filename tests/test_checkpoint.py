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
