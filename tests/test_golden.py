"""The committed fixtures in tests/golden/ (tools/make_golden.py): published PRNG vectors pin the
oracle; the oracle regression vectors must still be reproduced by the oracle."""
import json
from pathlib import Path

import numpy as np

from oracle import jaxrand as jr
from oracle import levels as olv
from oracle import rollout as oro
from oracle import sampler as osp

GOLD = Path(__file__).resolve().parent / "golden"


def test_published_prng_vectors():
    k = json.loads((GOLD / "prng_kat.json").read_text())
    for key, x, y in k["threefry2x32"]:
        out = jr.threefry2x32(key[0], key[1], x[0], x[1])
        assert [int(out[0]), int(out[1])] == y
    assert jr.split(jr.PRNGKey(0)).tolist() == k["split_PRNGKey0"]
    assert np.float32(jr.uniform(jr.PRNGKey(0))) == np.float32(k["uniform_PRNGKey0"])
    assert np.float32(jr.normal(jr.PRNGKey(0), ())) == np.float32(k["normal_PRNGKey0"])
    assert np.float32(jr.normal(jr.PRNGKey(42), ())) == np.float32(k["normal_PRNGKey42"])


def test_levels_fixture():
    g = np.load(GOLD / "levels.npz")
    for m in ("dense", "tabular", "all_shortlife", "mazes", "rand_all"):
        p, lt = olv.reset_env_params(g["keys"], m)
        assert np.array_equal(olv.pack_levels(p, lt, olv.env_spec(m)), g[m]), m


def test_rollout_fixture():
    g = np.load(GOLD / "rollout_dense.npz")
    spec = olv.env_spec("dense")
    p, _ = olv.reset_env_params(g["level_keys"], "dense")
    st = oro.batch_reset(spec, g["reset_keys"], p, 64)
    tr, _, cum = oro.batch_rollout(spec, g["roll_keys"], g["theta"], p, st, 20)
    assert np.array_equal(tr["action"], g["action"])
    assert np.array_equal(tr["idx"], g["idx"])
    assert np.array_equal(cum, g["cum"])


def test_plr_fixture():
    g = np.load(GOLD / "plr.npz")
    s, a, n, ks = g["score"], g["active"], g["new"], g["keys"]
    ids, _, _, _ = osp.reset_lowest_scoring(s, a, n, 512)
    assert np.array_equal(ids, g["reset_ids"])
    assert np.array_equal(osp.replay_ids(ks[1], s, a, n, 512, "rank"), g["rep_rank"])
    assert np.array_equal(osp.random_ids(ks[2], a, n, 512), g["rnd"])
