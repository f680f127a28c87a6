"""Writes tests/golden/: published jax PRNG known answers and oracle regression vectors.

    python tools/make_golden.py

* prng_kat.json — published vectors only (Random123 threefry2x32-20 KATs as used by jax's
  random_test; split/uniform/normal of PRNGKey(0)/(42) as printed in the JAX documentation).  These
  are the only externally pinned values for this path: the reference ships no tests or fixtures and
  jax is not installable here.
* levels.npz, rollout_dense.npz, plr.npz — vectors produced by the CPU restatement (oracle/) at
  fixed keys: regression fixtures so the device tests can check full-size outputs without re-running
  the oracle, and so an oracle change is visible in review.  They are NOT reference outputs.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from oracle import jaxrand as jr  # noqa: E402
from oracle import levels as olv  # noqa: E402
from oracle import rollout as oro  # noqa: E402
from oracle import sampler as osp  # noqa: E402

GOLD = ROOT / "tests" / "golden"
MODES = ["dense", "sparse", "long", "longer", "long_dense", "tabular", "all_shortlife", "all_vrandlife", "mazes",
         "small", "medium", "large", "debug", "rand_dense", "rand_small", "rand_all", "sixteen_rooms", "labyrinth"]


def main():
    GOLD.mkdir(parents=True, exist_ok=True)
    kat = {
        "source": "Random123 threefry2x32-20 KATs (jax random_test); JAX documentation examples",
        "threefry2x32": [[[0, 0], [0, 0], [0x6B200159, 0x99BA4EFE]],
                         [[0xFFFFFFFF, 0xFFFFFFFF], [0xFFFFFFFF, 0xFFFFFFFF], [0x1CB996FC, 0xBB002BE7]],
                         [[0x13198A2E, 0x03707344], [0x243F6A88, 0x85A308D3], [0xC4923A9C, 0x483DF7A0]]],
        "split_PRNGKey0": [[4146024105, 967050713], [2718843009, 1272950319]],
        "uniform_PRNGKey0": 0.41845703,
        "normal_PRNGKey0": -0.20584226,
        "normal_PRNGKey42": -0.18471177,
    }
    (GOLD / "prng_kat.json").write_text(json.dumps(kat, indent=1))
    keys = jr.split(jr.PRNGKey(2024), 16)
    lv = {"keys": keys}
    for m in MODES:
        spec = olv.env_spec(m)
        p, lt = olv.reset_env_params(keys, m)
        lv[m] = olv.pack_levels(p, lt, spec)
    np.savez_compressed(GOLD / "levels.npz", **lv)
    # one dense-mode rollout: 2 agents x 64 workers x 20 steps from a fixed actor
    mode, N, W, T = "dense", 2, 64, 20
    spec = olv.env_spec(mode)
    lk = jr.split(jr.PRNGKey(7), N)
    p, lt = olv.reset_env_params(lk, mode)
    theta = (np.random.RandomState(0).randn(N, spec.obs_dim, 5) * 2.0).astype(np.float32)
    rk = jr.split(jr.PRNGKey(8), N)
    st = oro.batch_reset(spec, rk, p, W)
    k2 = jr.split(jr.PRNGKey(9), N)
    tr, _, cum = oro.batch_rollout(spec, k2, theta, p, st, T)
    np.savez_compressed(GOLD / "rollout_dense.npz", level_keys=lk, reset_keys=rk, roll_keys=k2, theta=theta,
                        idx=tr["idx"], time=tr["time"], action=tr["action"].astype(np.int32), reward=tr["reward"],
                        done=tr["done"], cum=cum)
    # PLR buffer selection at B=4000, N=512
    rs = np.random.RandomState(3)
    B, Nn = 4000, 512
    score = (np.round(rs.randn(B) * 4) / 4).astype(np.float32)
    active = np.zeros(B, bool)
    active[rs.choice(B, Nn, replace=False)] = True
    new = (rs.rand(B) < 0.3) & ~active
    ks = jr.split(jr.PRNGKey(11), 3)
    ids, _, _, _ = osp.reset_lowest_scoring(score, active, new, Nn)
    rep = osp.replay_ids(ks[1], score, active, new, Nn, "rank")
    repp = osp.replay_ids(ks[1], score, active, new, Nn, "proportional")
    rnd = osp.random_ids(ks[2], active, new, Nn)
    ch, use = osp.select(ks[0], rep, rnd, active, new, Nn, 0.5)
    np.savez_compressed(GOLD / "plr.npz", score=score, active=active, new=new, keys=ks, reset_ids=ids, rep_rank=rep,
                        rep_prop=repp, rnd=rnd, chosen_rank=ch, use=use)
    print("wrote", sorted(x.name for x in GOLD.iterdir()))


if __name__ == "__main__":
    main()
