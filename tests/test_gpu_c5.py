"""C5's per-rank workload at full per-GPU size on one GPU (BASELINE configs[4]: env_mode=mazes, num_agents=4096
sharded over 8 x MI355X).

Rank r of 8 owns agents [512 r, 512 (r + 1)) of the 4096: every rank derives all 4096 per-agent keys
(meta/train.py:121 ``split(rng, num_agents)``, level_sampler.py:112-114,178 for the levels and agents) and keeps
its contiguous slice (util/jax.py:25-41 runs the agent axis as one vmapped batch per mini-batch).  Here the World
has size 8 but no process group, so the meta-gradient all-reduce is the identity and the step runs exactly the
rank's shard of the 8-GPU job: one full meta-step (K=5, W=64, T=20) of 512 mazes agents on the HIP path.

Checked against the oracle's slice of the 4096-key split:
  * the rank's 512 level records, bit-exact;
  * sampled agents' actor/critic/value-critic tables and env states, bit-exact;
  * rollout 0 of the meta-step for the sampled agents (indices, times, actions, rewards, dones), bit-exact;
  * the local meta-gradient finite and 203,946 long (mazes: no lifetime conditioning), metrics finite.
RCCL on hardware (the all-reduce across 8 GPUs) is not exercised here: the driver's 8-GPU node runs it.
"""
import numpy as np
import pytest
import torch

from oracle import agents as oag
from oracle import jaxrand as jr
from oracle import levels as olv
from oracle import rollout as oro

pytestmark = pytest.mark.gpu

N_TOTAL, WORLD = 4096, 8


@pytest.mark.parametrize("rank", [0, 7])
def test_c5_rank_shard_meta_step(rank):
    from test_gpu_env import _state_np
    from toued.dist import World
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = parse_args(["--env_mode", "mazes", "--num_agents", str(N_TOTAL), "--num_mini_batches", "1",
                       "--seed", "0"])
    tr = Trainer(args, World(rank=rank, size=WORLD))
    lo, hi, n = tr.sl
    assert (lo, hi, n) == (512 * rank, 512 * (rank + 1), N_TOTAL)
    ag = tr.agents
    assert ag.n == 512
    spec = olv.env_spec("mazes")
    D, W, T, K = spec.obs_dim, args.env_workers, args.train_rollout_len, args.num_agent_updates
    # ---- Trainer's key chain (train.py:20-31 -> level_sampler.py:103-132), the oracle's slice of each split
    rng = jr.PRNGKey(0)
    ks = jr.split(rng, 3)
    rng = ks[0]
    ks = jr.split(rng, 2)
    rng, sub = ks[0], ks[1]
    r2 = jr.split(sub, 2)                          # random branch: (rng, sub) = split(rng)
    lkeys = jr.split(r2[1], N_TOTAL)[lo:hi]
    r3 = jr.split(r2[0], 2)
    akeys = jr.split(r3[1], N_TOTAL)[lo:hi]
    r4 = jr.split(r3[0], 2)
    vkeys = jr.split(r4[1], N_TOTAL)[lo:hi]
    p, lt = olv.reset_env_params(lkeys, "mazes")
    lv_ref = olv.pack_levels(p, lt, spec)
    lv_dev = ag.levels.cpu().numpy()
    np.testing.assert_array_equal(lv_dev, lv_ref, err_msg="level records of the rank's slice")
    sel = np.array([0, 1, 255, 511])
    th0 = ag.theta.cpu().numpy()
    ph0 = ag.phi.cpu().numpy()
    vc0 = ag.vcrit.cpu().numpy()
    state0 = ag.state.cpu().numpy()
    cols = np.concatenate([np.arange(a * W, (a + 1) * W) for a in sel])
    ps = {k: v[sel] for k, v in p.items()}
    ost0 = oro.batch_reset(spec, jr.split(akeys[sel], 2)[:, 0], ps, W)
    gst = _state_np(torch.from_numpy(state0[:, cols]), spec)
    for k in ("time", "pos", "obj_existss", "early_term", "obj_poss"):
        np.testing.assert_array_equal(gst[k], ost0[k], err_msg=f"initial env state {k}")
    for j, a in enumerate(sel):
        t_ref, c_ref = oag.create_agent(jr.split(akeys[a], 2)[1], D, 8)
        np.testing.assert_array_equal(th0[a], t_ref, err_msg=f"actor table {a}")
        np.testing.assert_array_equal(ph0[a], c_ref, err_msg=f"critic table {a}")
        np.testing.assert_array_equal(vc0[a], oag.lecun_table(vkeys[a], D, 1).reshape(vc0[a].shape),
                                      err_msg=f"value critic {a}")
    # ---- one full meta-step of the shard (train.py:36-54): LPG meta-gradient step, then level_sampler.sample
    mk = jr.split(rng, 2)
    metrics = tr.meta_step()
    torch.cuda.synchronize()
    step = tr.step_fn
    g = step.grad
    assert g.numel() == 203946 and bool(torch.isfinite(g).all()) and float(g.abs().sum()) > 0
    for key, v in metrics.items():
        if isinstance(v, dict):
            for k2, v2 in v.items():
                assert bool(torch.isfinite(torch.as_tensor(v2)).all()), (key, k2)
        else:
            assert bool(torch.isfinite(torch.as_tensor(v)).all()), key
    assert bool(torch.isfinite(tr.eta).all())
    # rollout 0: (r0, t) = split(key_a) (meta/train.py:41), (t, roll_0) = split(t) (lpg_agent.py:107)
    keys_a = jr.split(mk[1], N_TOTAL)[lo:hi][sel]
    t0 = jr.split(keys_a, 2)[:, 1]
    roll0 = jr.split(t0, 2)[:, 1]
    otr, _, _ = oro.batch_rollout(spec, roll0, th0[sel], ps, ost0, T)
    trj = step.traj
    for name, got in (("idx", trj.obs_idx), ("time", trj.obs_time), ("action", trj.action), ("reward", trj.reward),
                      ("done", trj.done)):
        gk = got[0].cpu().numpy()[sel]
        np.testing.assert_array_equal(gk, otr[name].transpose(0, 2, 1).astype(gk.dtype), err_msg=f"rollout 0 {name}")
    assert K == 5
