"""Device outputs vs the committed fixtures in tests/golden/ (bit-exact; no oracle at run time)."""
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


def dk(a):
    from toued.prng import from_uint32_numpy
    return from_uint32_numpy(np.asarray(a, np.uint32), "cuda")


def test_levels_golden():
    from toued.env import LevelGenerator
    g = np.load(GOLD / "levels.npz")
    for m in [k for k in g.files if k != "keys"]:
        assert np.array_equal(LevelGenerator(m)(dk(g["keys"])).cpu().numpy(), g[m]), m


def test_rollout_golden():
    from toued.env import LevelGenerator
    from toued.rollout import RolloutWrapper
    g = np.load(GOLD / "rollout_dense.npz")
    levels = LevelGenerator("dense")(dk(g["level_keys"]))
    ro = RolloutWrapper("dense", 20, env_workers=64)
    (_, _), st = ro.batch_reset(dk(g["reset_keys"]), levels)
    tr, _, cum = ro.batch_rollout(dk(g["roll_keys"]), torch.from_numpy(g["theta"]).cuda(), levels, st)
    assert np.array_equal(tr.action.cpu().numpy(), g["action"].transpose(0, 2, 1))
    assert np.array_equal(tr.obs_idx.cpu().numpy(), g["idx"].transpose(0, 2, 1))
    assert np.array_equal(tr.reward.cpu().numpy(), g["reward"].transpose(0, 2, 1))
    assert np.array_equal(cum.cpu().numpy(), g["cum"])


def test_plr_golden():
    from toued import _lib
    g = np.load(GOLD / "plr.npz")
    s, a, n = (torch.from_numpy(g[k]).cuda() for k in ("score", "active", "new"))
    ids = torch.empty(512, dtype=torch.int32, device="cuda")
    _lib.call("toued_plr_reset_ids", 4000, 512, _lib.ptr(s), _lib.ptr(a), _lib.ptr(n), _lib.ptr(ids),
              _lib.stream_ptr())
    assert np.array_equal(ids.cpu().numpy(), g["reset_ids"])
    ks = g["keys"]
    kbuf = dk(np.stack([ks[1], ks[2], ks[0]]))
    for prop, rep_key in ((0, "rep_rank"), (1, "rep_prop")):
        out = [torch.empty(512, dtype=torch.int32, device="cuda") for _ in range(4)]
        _lib.call("toued_plr_sample", 4000, 512, _lib.ptr(s), _lib.ptr(a), _lib.ptr(n), _lib.ptr(kbuf), prop, 1.0,
                  0.5, *[_lib.ptr(o) for o in out], _lib.stream_ptr())
        assert np.array_equal(out[1].cpu().numpy(), g[rep_key])
        assert np.array_equal(out[2].cpu().numpy(), g["rnd"])
        if prop == 0:
            assert np.array_equal(out[0].cpu().numpy(), g["chosen_rank"])
            assert np.array_equal(out[3].cpu().numpy().astype(bool), g["use"])
