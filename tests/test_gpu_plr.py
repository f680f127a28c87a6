"""GPU parity of the GROOVE / PLR path: A2C antagonist, algorithmic regret, level buffer.

  * agent tables (flax lecun_normal with flax's param-key derivation): bit-exact vs oracle/agents.py
  * one A2C update (agents/a2c.py:19-76): the rollout bit-exact, the updated actor/critic within
    float32-vs-float64 tolerance of the torch autograd oracle (oracle/a2c.py):
    relative L2 error of the parameter change < 1e-4
  * key plumbing of _compute_algorithmic_regret with max_lifetime=0 (untrained antagonist):
    regret within 1e-5 of the oracle (float32 mean over workers vs float64)
  * regret with TRAINED antagonists (all_shortlife / mazes, 3-4 A2C updates, fused and unfused): each
    update's rollout bit-exact and parameter change within 2e-5 of float64 autograd, regret within 1e-5;
    and at full C3 size (N=512, 250 updates) batch-invariance plus the oracle eval of 4 agents
  * buffer logic (level_sampler.py:169-234, 331-408): reset ids, replay ids (rank and
    proportional), random ids, replay/random selection — bit-exact vs oracle/sampler.py
  * LevelSampler.sample end to end (alg_regret): buffer flags and chosen levels bit-exact vs the
    oracle driven by the device's regret scores
"""
import numpy as np
import pytest
import torch

from oracle import a2c as oa2c
from oracle import agents as oag
from oracle import jaxrand as jr
from oracle import levels as olv
from oracle import meta as ometa
from oracle import rollout as oro
from oracle import sampler as osp

pytestmark = pytest.mark.gpu


def dk(a):
    from toued.prng import from_uint32_numpy
    return from_uint32_numpy(a, "cuda")


def _ahyp(mode):
    from toued.agents import AgentHyperparams
    from toued.env import get_agent_hypers
    return AgentHyperparams(**get_agent_hypers(mode), critic_dims=1)


def _ost(state0, nmax):
    ex = np.stack([(state0[2] >> i) & 1 for i in range(nmax)], 1).astype(bool)
    return {"time": state0[0], "pos": state0[1], "obj_existss": ex, "early_term": state0[3].astype(bool),
            "obj_poss": state0[4:4 + nmax].T.copy()}


@pytest.mark.parametrize("mode,cols", [("dense", 5), ("all_shortlife", 1), ("mazes", 8)])
def test_init_tables_bitexact(mode, cols):
    from toued.agents import lecun_tables
    spec = olv.env_spec(mode)
    D = spec.obs_dim
    keys = jr.split(jr.PRNGKey(11), 3)
    got = lecun_tables(dk(keys), D, cols).cpu().numpy()
    for a in range(3):
        assert np.array_equal(got[a], oag.lecun_table(keys[a], D, cols)), a


def _a2c_setup(mode, N, W, T, seed=0, scale=20.0):
    from toued.agents import create_agents
    from toued.env import LevelGenerator
    from toued.rollout import RolloutWrapper
    keys = jr.split(jr.PRNGKey(seed), N)
    levels = LevelGenerator(mode)(dk(keys))
    p, lt = olv.reset_env_params(keys, mode)
    ro = RolloutWrapper(mode, T, env_workers=W)
    D = ro.obs_dim
    theta, vc = create_agents(dk(jr.split(jr.PRNGKey(seed + 1), N)), D, 1)
    theta.mul_(scale)
    vcrit = (vc.reshape(N, D) * scale).contiguous()
    (_, _), state = ro.batch_reset(dk(jr.split(jr.PRNGKey(seed + 2), N)), levels)
    return ro, levels, p, lt, theta, vcrit, state, D


@pytest.mark.parametrize("fused", [True, False])
def test_a2c_update_matches_oracle(fused):
    """fused: the LDS-table update kernel (toued_a2c_update); else toued_a2c_grad + toued_a2c_apply."""
    from toued.a2c import A2CHyperparams, A2CTrainer
    mode, N, W, T = "dense", 3, 64, 20
    ro, levels, p, lt, theta, vcrit, state, D = _a2c_setup(mode, N, W, T)
    spec = olv.env_spec(mode)
    th0, vc0, st0 = theta.cpu().numpy(), vcrit.cpu().numpy(), state.cpu().numpy()
    rng = jr.split(jr.PRNGKey(9), N)
    # one launch per update (the chain kernel keeps its trajectories in LDS; its parity with this path:
    # test_a2c_chain_matches_launch_per_update)
    tr = A2CTrainer(ro, A2CHyperparams(), _ahyp(mode), use_graph=False, fused=fused, chain=False)
    step = torch.zeros(N, dtype=torch.int32, device="cuda")
    loss = tr.train(dk(rng), theta, vcrit, step, levels, state, 1).cpu().numpy()
    b = tr._bufs["tr"]
    idx, tm, act = b.obs_idx.cpu().numpy(), b.obs_time.cpu().numpy(), b.action.cpu().numpy()
    rew, dn = b.reward.cpu().numpy(), b.done.cpu().numpy()
    # rollout of update 0 with key split(rng)[1], bit-exact
    sub = jr.split(rng, 2)[:, 1]
    otr, _, _ = oro.batch_rollout(spec, sub, th0, p, _ost(st0, spec.max_n_objs), T)
    assert np.array_equal(act, otr["action"].transpose(0, 2, 1))
    assert np.array_equal(idx, otr["idx"].transpose(0, 2, 1))
    assert np.array_equal(rew, otr["reward"].transpose(0, 2, 1))
    assert step.cpu().numpy().tolist() == [1] * N
    th1, vc1 = theta.cpu().numpy(), vcrit.cpu().numpy()
    hyp = ometa.Hypers()
    for a in range(N):
        traj = {"idx": idx[a].T.copy(), "time": tm[a].T.copy(), "action": act[a].T.astype(np.int64),
                "reward": rew[a].T.copy(), "done": dn[a].T.astype(bool)}
        t_ref, v_ref, s_ref, al, cl = oa2c.a2c_step(
            torch.from_numpy(th0[a].astype(np.float64)), torch.from_numpy(vc0[a][:, None].astype(np.float64)), 0,
            int(lt[a]), traj, hyp, 40.0, 4.0, 0.5)
        dt_ref = t_ref.numpy() - th0[a]
        dv_ref = v_ref.numpy()[:, 0] - vc0[a]
        dt = th1[a].astype(np.float64) - th0[a]
        dv = vc1[a].astype(np.float64) - vc0[a]
        assert np.linalg.norm(dt - dt_ref) <= 1e-4 * np.linalg.norm(dt_ref) + 1e-6, a
        assert np.linalg.norm(dv - dv_ref) <= 1e-4 * np.linalg.norm(dv_ref) + 1e-6, a
        assert abs(loss[a, 0] - al) <= 1e-4 * max(1.0, abs(al))
        assert abs(loss[a, 1] - cl) <= 1e-4 * max(1.0, abs(cl))


def test_a2c_graph_replay_matches_eager_and_lifetime_discard():
    from toued.a2c import A2CHyperparams, A2CTrainer
    from toued.env import L_LIFETIME
    mode, N, W, T, U = "dense", 4, 64, 20, 5
    ro, levels, p, lt, theta, vcrit, state, D = _a2c_setup(mode, N, W, T, seed=3)
    levels[:, L_LIFETIME] = torch.tensor([1, 3, 100, 5], dtype=torch.int32, device="cuda")
    rng = dk(jr.split(jr.PRNGKey(5), N))
    outs = []
    for g in (False, True):
        th, vc, st = theta.clone(), vcrit.clone(), state.clone()
        step = torch.zeros(N, dtype=torch.int32, device="cuda")
        tr = A2CTrainer(ro, A2CHyperparams(), _ahyp(mode), use_graph=g)
        tr.train(rng, th, vc, step, levels, st, U)
        if g:   # a second replay of the captured graph on fresh inputs gives the same answer
            th2, vc2, st2 = theta.clone(), vcrit.clone(), state.clone()
            step2 = torch.zeros(N, dtype=torch.int32, device="cuda")
            tr.train(rng, th2, vc2, step2, levels, st2, U)
            torch.testing.assert_close(th2, th, rtol=1e-5, atol=1e-6)
        outs.append((th, vc, st, step))
    (th_e, vc_e, st_e, s_e), (th_g, vc_g, st_g, s_g) = outs
    assert s_e.cpu().tolist() == [1, 3, 5, 5]
    assert torch.equal(s_e, s_g)
    torch.testing.assert_close(th_g, th_e, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(vc_g, vc_e, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("self_draws", ["0", "1"])
@pytest.mark.parametrize("mode,W,U", [("dense", 64, 40), ("all_shortlife", 32, 7), ("mazes", 64, 33)])
def test_a2c_chain_matches_launch_per_update(mode, W, U, self_draws, monkeypatch):
    """toued_a2c_chain (the whole update chain in one kernel per 32 updates, trajectories in LDS) against one
    toued_rollout_env + one toued_a2c_update launch per update: actor/critic tables, env state, step counters (with
    lifetime discards) and losses bit-identical, over several draw chunks and a partial last chunk.  self_draws = 1:
    toued_a2c_chain_self (one launch, the draws made in the env chain's idle waves)."""
    from toued.a2c import A2CHyperparams, A2CTrainer
    from toued.env import L_LIFETIME
    monkeypatch.setenv("TOUED_A2C_SELF", self_draws)
    N, T = 4, 20
    ro, levels, p, lt, theta, vcrit, state, D = _a2c_setup(mode, N, W, T, seed=31)
    levels[:, L_LIFETIME] = torch.tensor([1, U // 2, 1000, U - 1], dtype=torch.int32, device="cuda")
    rng = dk(jr.split(jr.PRNGKey(37), N))
    outs = []
    for chain in (False, True):
        th, vc, st = theta.clone(), vcrit.clone(), state.clone()
        step = torch.zeros(N, dtype=torch.int32, device="cuda")
        tr = A2CTrainer(ro, A2CHyperparams(), _ahyp(mode), use_graph=False, chain=chain)
        assert tr.use_chain(W, T, D) == chain
        assert tr.use_self_draws(W, T, D) == (self_draws == "1")
        loss = tr.train(rng, th, vc, step, levels, st, U)
        outs.append((th, vc, st, step, loss))
    for x, y, name in zip(outs[0], outs[1], ("theta", "vcrit", "state", "step", "loss")):
        assert torch.equal(x, y), name
    assert outs[1][3].cpu().tolist() == [1, U // 2, U, U - 1]


def test_a2c_c1_tabular_n8_matches_oracle():
    """BASELINE config C1: the A2C-only inner loop (train_a2c_agent, agents/a2c.py:79-125) on env_mode=tabular
    (the defined manual dispatch over the five LPG tabular levels, D = 5409 padded) with num_agents = 8 and the
    mode's agent hyperparameters (configs.py:322-325 via get_agent_hypers).  Five updates, every update's
    rollout bit-exact from the oracle's own key chain (a2c.py:97) and the carried env state, every parameter
    change within 2e-5 of float64 autograd (oracle/a2c.py); the step counters and lifetime discard likewise."""
    from toued.a2c import A2CHyperparams, A2CTrainer
    from toued.env import get_agent_hypers
    mode, N, W, T, U = "tabular", 8, 64, 20, 5
    ro, levels, p, lt, theta, vcrit, state, D = _a2c_setup(mode, N, W, T, seed=21)
    spec = olv.env_spec(mode)
    assert D == spec.obs_dim and D > 5000
    ah = get_agent_hypers(mode)
    st0 = state.cpu().numpy()
    rng = jr.split(jr.PRNGKey(23), N)
    inputs = (theta.clone(), vcrit.clone(), state.clone())
    tr = A2CTrainer(ro, A2CHyperparams(), _ahyp(mode))
    tr.record = []
    step = torch.zeros(N, dtype=torch.int32, device="cuda")
    tr.train(dk(rng), theta, vcrit, step, levels, state, U)
    assert len(tr.record) == U
    # the production path (graph-replayed update chain) gives the recorded eager chain's tables bit for bit
    th_g, vc_g, st_g = inputs
    step_g = torch.zeros(N, dtype=torch.int32, device="cuda")
    A2CTrainer(ro, A2CHyperparams(), _ahyp(mode)).train(dk(rng), th_g, vc_g, step_g, levels, st_g, U)
    assert torch.equal(th_g, theta) and torch.equal(vc_g, vcrit) and torch.equal(st_g, state)
    assert step.cpu().tolist() == step_g.cpu().tolist()
    ost = _a2c_follow(spec, p, lt, tr.record, rng, _ost(st0, spec.max_n_objs),
                      lrs=(ah["actor_learning_rate"], ah["critic_learning_rate"], ah["max_grad_norm"]))
    from test_gpu_env import _assert_state
    _assert_state(state, ost, spec)
    assert torch.equal(theta, tr.record[-1]["theta_out"])


@pytest.mark.parametrize("mode", ["mazes", "dense"])
def test_regret_untrained_matches_oracle(mode):
    """max_lifetime = 0: regret = eval(fresh A2C actor) - eval(LPG actor) — checks the key
    derivation of _compute_algorithmic_regret, agent creation and eval_agent."""
    from toued.agents import create_agents
    from toued.env import LevelGenerator
    from toued.parse_args import parse_args
    from toued.level_sampler import LevelSampler
    from toued.plr import algorithmic_regret
    N = 3
    args = parse_args(["--env_mode", mode, "--score_function", "alg_regret", "--num_agents", str(N), "--num_mini_batches", "1"])
    smp = LevelSampler(args)
    smp.max_lifetime = 0
    spec = olv.env_spec(mode)
    lk = jr.split(jr.PRNGKey(21), N)
    levels = LevelGenerator(mode)(dk(lk))
    p, _ = olv.reset_env_params(lk, mode)
    D = spec.obs_dim
    lpg_theta, _ = create_agents(dk(jr.split(jr.PRNGKey(22), N)), D, 8)
    lpg_theta.mul_(10.0)
    keys = jr.split(jr.PRNGKey(23), N)
    got = algorithmic_regret(smp, dk(keys), levels, lpg_theta).cpu().numpy()
    # oracle
    k = jr.split(keys, 2)
    rng, c = k[:, 0], k[:, 1]
    ag = jr.split(c, 2)[:, 1]
    a2c_theta = np.stack([oag.create_agent(ag[a], D, 1)[0] for a in range(N)])
    rng = jr.split(rng, 2)[:, 0]
    ev = jr.split(rng, 2)
    L = smp.max_rollout_len
    r_lpg = oag.eval_agent(spec, ev[:, 0], p, lpg_theta.cpu().numpy(), 64, L)
    r_a2c = oag.eval_agent(spec, ev[:, 1], p, a2c_theta, 64, L)
    np.testing.assert_allclose(got, r_a2c - r_lpg, atol=1e-5, rtol=0)


def _a2c_follow(spec, p, lt, rec, keys_tr, ost, tol=2e-5, lrs=(40.0, 4.0, 0.5)):
    """Replays a recorded A2C chain (A2CTrainer.record) on the oracle: every update's rollout bit-exact from
    the device's starting tables and the oracle's own key chain (a2c.py:97 rng, _rng = split(rng)) and carried
    env state; every update's parameter change within `tol` relative L2 of the float64 autograd oracle
    (oracle/a2c.py) applied to the same starting tables.  Returns the oracle end state."""
    hyp = ometa.Hypers()
    tr = keys_tr
    for u, r in enumerate(rec):
        s2 = jr.split(tr, 2)
        tr, sub = s2[:, 0], s2[:, 1]
        th0 = r["theta"].cpu().numpy()
        otr, ost, _ = oro.batch_rollout(spec, sub, th0, p, ost, 20)
        b = r["traj"]
        idx, tm, act = b.obs_idx.cpu().numpy(), b.obs_time.cpu().numpy(), b.action.cpu().numpy()
        rew, dn = b.reward.cpu().numpy(), b.done.cpu().numpy()
        for name, got in (("idx", idx), ("time", tm), ("action", act), ("reward", rew), ("done", dn)):
            np.testing.assert_array_equal(got, otr[name].transpose(0, 2, 1).astype(got.dtype),
                                          err_msg=f"update {u} {name}")
        vc0, st0 = r["vcrit"].cpu().numpy(), r["step"].cpu().numpy()
        th1, vc1, st1 = r["theta_out"].cpu().numpy(), r["vcrit_out"].cpu().numpy(), r["step_out"].cpu().numpy()
        for a in range(th0.shape[0]):
            traj = {"idx": idx[a].T.copy(), "time": tm[a].T.copy(), "action": act[a].T.astype(np.int64),
                    "reward": rew[a].T.copy(), "done": dn[a].T.astype(bool)}
            t_ref, v_ref, s_ref, _, _ = oa2c.a2c_step(
                torch.from_numpy(th0[a].astype(np.float64)), torch.from_numpy(vc0[a][:, None].astype(np.float64)),
                int(st0[a]), int(lt[a]), traj, hyp, *lrs)
            assert int(st1[a]) == s_ref, (u, a)
            dt_ref, dv_ref = t_ref.numpy() - th0[a], v_ref.numpy()[:, 0] - vc0[a]
            dt, dv = th1[a].astype(np.float64) - th0[a], vc1[a].astype(np.float64) - vc0[a]
            assert np.linalg.norm(dt - dt_ref) <= tol * np.linalg.norm(dt_ref) + 1e-7, (u, a)
            assert np.linalg.norm(dv - dv_ref) <= tol * np.linalg.norm(dv_ref) + 1e-7, (u, a)
    return ost


@pytest.mark.parametrize("mode,max_lifetime,fused", [("all_shortlife", 4, None), ("all_shortlife", 3, False),
                                                     ("mazes", 3, None)])
def test_regret_trained_antagonist_matches_oracle(mode, max_lifetime, fused):
    """_compute_algorithmic_regret (level_sampler.py:293-329) with a TRAINED antagonist: train_a2c_agent
    (a2c.py:79-125) for max_lifetime updates.  Checked against the oracle link by link: the antagonist's
    initial tables bit-exact (flax lecun init), every A2C update's rollout bit-exact and its parameter change
    within 2e-5 of float64 autograd, then regret = eval(trained A2C) - eval(LPG) within 1e-5 with both eval
    rollouts regenerated by the oracle from the oracle's keys."""
    from toued.agents import create_agents
    from toued.env import LevelGenerator
    from toued.level_sampler import LevelSampler
    from toued.parse_args import parse_args
    from toued.plr import algorithmic_regret
    N = 3
    args = parse_args(["--env_mode", mode, "--score_function", "alg_regret", "--num_agents", str(N),
                       "--num_mini_batches", "1"])
    smp = LevelSampler(args)
    smp.max_lifetime = max_lifetime
    trn = smp.a2c_trainer()
    trn.fused = fused
    trn.record = []
    spec = olv.env_spec(mode)
    lk = jr.split(jr.PRNGKey(31), N)
    levels = LevelGenerator(mode)(dk(lk))
    p, lt = olv.reset_env_params(lk, mode)
    D = spec.obs_dim
    lpg_theta, _ = create_agents(dk(jr.split(jr.PRNGKey(32), N)), D, 8)
    lpg_theta.mul_(10.0)
    keys = jr.split(jr.PRNGKey(33), N)
    got = algorithmic_regret(smp, dk(keys), levels, lpg_theta).cpu().numpy()
    rec = trn.record
    assert len(rec) == max_lifetime
    # oracle key chain of _compute_algorithmic_regret / _create_agent (level_sampler.py:273-329)
    k = jr.split(keys, 2)
    rng, c = k[:, 0], k[:, 1]
    wc = jr.split(c, 2)
    w_rng, ag_rng = wc[:, 0], wc[:, 1]
    ost = oro.batch_reset(spec, w_rng, p, smp.env_workers)
    init = [oag.create_agent(ag_rng[a], D, 1) for a in range(N)]
    assert np.array_equal(rec[0]["theta"].cpu().numpy(), np.stack([x[0] for x in init]))
    assert np.array_equal(rec[0]["vcrit"].cpu().numpy(), np.stack([x[1][:, 0] for x in init]))
    k = jr.split(rng, 2)
    rng, tr = k[:, 0], k[:, 1]
    _a2c_follow(spec, p, lt, rec, tr, ost)
    theta_K = rec[-1]["theta_out"].cpu().numpy()
    assert not np.array_equal(theta_K, rec[0]["theta"].cpu().numpy())
    ev = jr.split(rng, 2)
    L = smp.max_rollout_len
    r_lpg = oag.eval_agent(spec, ev[:, 0], p, lpg_theta.cpu().numpy(), 64, L)
    r_a2c = oag.eval_agent(spec, ev[:, 1], p, theta_K, 64, L)
    np.testing.assert_allclose(got, r_a2c - r_lpg, atol=1e-5, rtol=0)


def test_a2c_chain_full_size_matches_launch_per_update():
    """C3's antagonist training at full size (512 all_shortlife antagonists x max_lifetime = 250 updates: eight chain
    launches, the last one partial, draws double-buffered on the side stream) bit-identical to one toued_rollout_env +
    one toued_a2c_update launch per update: tables, step counters, env state and the mean losses."""
    from toued.a2c import A2CHyperparams, A2CTrainer
    mode, N, W, T, U = "all_shortlife", 512, 64, 20, 250
    ro, levels, p, lt, theta, vcrit, state, D = _a2c_setup(mode, N, W, T, seed=51, scale=1.0)
    rng = dk(jr.split(jr.PRNGKey(53), N))
    outs = []
    for chain in (False, True):
        th, vc, st = theta.clone(), vcrit.clone(), state.clone()
        step = torch.zeros(N, dtype=torch.int32, device="cuda")
        tr = A2CTrainer(ro, A2CHyperparams(), _ahyp(mode), chain=chain)
        assert tr.use_chain(W, T, D) == chain
        loss = tr.train(rng, th, vc, step, levels, st, U)
        torch.cuda.synchronize()
        outs.append((th, vc, st, step, loss))
    for x, y, name in zip(outs[0], outs[1], ("theta", "vcrit", "state", "step", "loss")):
        assert torch.equal(x, y), name
    assert int(outs[1][3].max()) <= U and int(outs[1][3].min()) >= 1


def test_regret_full_size_batch_invariant():
    """C3 at full size: N=512 all_shortlife antagonists trained for the mode's max_lifetime (250) updates in
    one batch (graph-replayed fused kernels).  Size-independent properties: every score finite; the regret of
    an agent depends only on its own key, level and actor — re-scoring 4 of them alone gives bit-identical
    scores; and the eval part is the oracle's: with the device's trained tables of those 4, the oracle eval
    rollouts reproduce the regret within 1e-5."""
    from toued import prng
    from toued.agents import create_agents
    from toued.env import LevelGenerator
    from toued.level_sampler import LevelSampler
    from toued.parse_args import parse_args
    from toued.plr import algorithmic_regret
    mode, N = "all_shortlife", 512
    args = parse_args(["--env_mode", mode, "--score_function", "alg_regret", "--num_agents", str(N),
                       "--num_mini_batches", "1"])
    smp = LevelSampler(args)
    assert smp.max_lifetime == 250
    lk = jr.split(jr.PRNGKey(41), N)
    levels = LevelGenerator(mode)(dk(lk))
    D = smp.obs_dim
    lpg_theta, _ = create_agents(dk(jr.split(jr.PRNGKey(42), N)), D, 8)
    lpg_theta.mul_(10.0)
    keys = dk(jr.split(jr.PRNGKey(43), N))
    full = algorithmic_regret(smp, keys, levels, lpg_theta)
    torch.cuda.synchronize()
    assert torch.isfinite(full).all()
    assert (full.abs() > 0).any()
    sel = torch.tensor([0, 77, 300, 511], device="cuda")
    part = algorithmic_regret(smp, keys[sel].contiguous(), levels[sel].contiguous(), lpg_theta[sel].contiguous())
    assert torch.equal(part, full[sel])
    # oracle eval of the same 4 from the trained tables of an eager re-run (record hook) of the 4-agent batch
    trn = smp.a2c_trainer()
    trn.record = []
    again = algorithmic_regret(smp, keys[sel].contiguous(), levels[sel].contiguous(), lpg_theta[sel].contiguous())
    assert torch.equal(again, part)
    theta_K = trn.record[-1]["theta_out"].cpu().numpy()
    trn.record = None
    kk = prng.to_uint32_numpy(keys[sel])
    p, _ = olv.reset_env_params(lk[sel.cpu().numpy()], mode)
    spec = olv.env_spec(mode)
    rng = jr.split(jr.split(kk, 2)[:, 0], 2)[:, 0]
    ev = jr.split(rng, 2)
    r_lpg = oag.eval_agent(spec, ev[:, 0], p, lpg_theta[sel].cpu().numpy(), 64, smp.max_rollout_len)
    r_a2c = oag.eval_agent(spec, ev[:, 1], p, theta_K, 64, smp.max_rollout_len)
    np.testing.assert_allclose(part.cpu().numpy(), r_a2c - r_lpg, atol=1e-5, rtol=0)


def _buffer_state(B, N, seed, n_active, frac_new, ties=True):
    rs = np.random.RandomState(seed)
    score = rs.randn(B).astype(np.float32)
    if ties:
        score = (np.round(score * 4) / 4).astype(np.float32)
        score[rs.rand(B) < 0.05] = -0.0
    active = np.zeros(B, bool)
    active[rs.choice(B, n_active, replace=False)] = True
    new = (rs.rand(B) < frac_new) & ~active
    return score, active, new


@pytest.mark.parametrize("B,N", [(4000, 512), (64, 8), (1000, 1000), (33, 7)])
def test_plr_reset_ids_bitexact(B, N):
    score, active, new = _buffer_state(B, N, B + N, min(N // 2, B), 0.3)
    ids = torch.empty(N, dtype=torch.int32, device="cuda")
    from toued import _lib
    s, a, n = (torch.from_numpy(x).cuda() for x in (score, active, new))
    _lib.call("toued_plr_reset_ids", B, N, _lib.ptr(s), _lib.ptr(a), _lib.ptr(n), _lib.ptr(ids), _lib.stream_ptr())
    ref, _, _, _ = osp.reset_lowest_scoring(score, active, new, N)
    assert np.array_equal(ids.cpu().numpy(), ref)


@pytest.mark.parametrize("transform", ["rank", "proportional"])
@pytest.mark.parametrize("B,N,n_active,frac_new", [(4000, 512, 512, 0.3), (4000, 512, 512, 0.9),
                                                    (300, 64, 32, 0.5), (100, 16, 0, 0.0)])
def test_plr_sample_bitexact(transform, B, N, n_active, frac_new):
    from toued import _lib
    score, active, new = _buffer_state(B, N, B * 7 + N, n_active, frac_new)
    if frac_new == 0.0:   # no new levels at all: the random draw sees p = 0/0
        new[:] = False
    keys = jr.split(jr.PRNGKey(B + N), 3)
    kbuf = np.stack([keys[1], keys[2], keys[0]])
    s, a, n = (torch.from_numpy(x).cuda() for x in (score, active, new))
    out = [torch.empty(N, dtype=torch.int32, device="cuda") for _ in range(4)]
    _lib.call("toued_plr_sample", B, N, _lib.ptr(s), _lib.ptr(a), _lib.ptr(n), _lib.ptr(dk(kbuf)),
              int(transform == "proportional"), 1.0, 0.5, *[_lib.ptr(o) for o in out], _lib.stream_ptr())
    chosen, rep, rnd, use = (o.cpu().numpy() for o in out)
    rep_ref = osp.replay_ids(keys[1], score, active, new, N, transform, 1.0)
    rnd_ref = osp.random_ids(keys[2], active, new, N)
    ch_ref, use_ref = osp.select(keys[0], rep_ref, rnd_ref, active, new, N, 0.5)
    assert np.array_equal(rep, rep_ref)
    assert np.array_equal(rnd, rnd_ref)
    assert np.array_equal(use.astype(bool), use_ref)
    assert np.array_equal(chosen, ch_ref)


def test_level_sampler_alg_regret_end_to_end():
    from toued import prng
    from toued.env import L_BUFID, L_LIFETIME
    from toued.level_sampler import LevelSampler
    from toued.parse_args import parse_args
    N, B = 8, 64
    args = parse_args(["--env_mode", "mazes", "--score_function", "alg_regret", "--num_agents", str(N), "--num_mini_batches", "1",
                       "--buffer_size", str(B)])
    smp = LevelSampler(args)
    smp.max_lifetime = 3
    buf = smp.initialize_buffer(prng.PRNGKey(0, "cuda"))
    buf, agents = smp.initial_sample(prng.PRNGKey(1, "cuda"), buf, N, False)
    assert buf.active.sum().item() == N
    # a first round with all agents terminated fills the buffer with scores
    agents.step = agents.levels[:, L_LIFETIME].clone()
    rng = prng.PRNGKey(2, "cuda")
    for it in range(3):
        pre = {k: getattr(buf, k).clone() for k in ("score", "active", "new", "levels")}
        term = (agents.step >= agents.levels[:, L_LIFETIME]).cpu().numpy()
        old_ids = agents.levels[:, L_BUFID].cpu().numpy()
        rng_np = prng.to_uint32_numpy(rng)
        buf, agents = smp.sample(rng, buf, agents)
        rng = prng.split(rng, 2)[1].contiguous()
        # oracle replay of the buffer logic with the device's regret scores
        r, sub = jr.split(rng_np, 2)
        sub_reset = sub
        ids, score, active, new = osp.reset_lowest_scoring(pre["score"].cpu().numpy(), pre["active"].cpu().numpy(),
                                                           pre["new"].cpu().numpy(), N)
        r, sub = jr.split(r, 2)
        sc = smp.last_plr["score"].cpu().numpy()
        score[old_ids[term]] = sc[term]
        active[old_ids[term]] = False
        new[old_ids[term]] = False
        k3 = jr.split(r, 3)
        rep = osp.replay_ids(k3[1], score, active, new, N, "rank", 1.0)
        rnd = osp.random_ids(k3[2], active, new, N)
        ch, _ = osp.select(k3[0], rep, rnd, active, new, N, 0.5)
        new_ids = np.where(term, ch, old_ids)
        active[new_ids] = True
        assert np.array_equal(buf.levels[torch.from_numpy(ids).long().cuda(), L_BUFID].cpu().numpy(), ids)
        # the reset levels themselves: gen(split(sub, N)) of the reset key (read on the side stream)
        p_new, lt_new = olv.reset_env_params(jr.split(sub_reset, N), "mazes")
        ref_new = olv.pack_levels(p_new, lt_new, olv.env_spec("mazes"), buffer_id=ids)
        assert np.array_equal(buf.levels[torch.from_numpy(ids).long().cuda()].cpu().numpy(), ref_new), it
        assert np.array_equal(buf.score.cpu().numpy(), score), it
        assert np.array_equal(buf.active.cpu().numpy(), active), it
        assert np.array_equal(buf.new.cpu().numpy(), new), it
        assert np.array_equal(agents.levels[:, L_BUFID].cpu().numpy(), new_ids), it
        assert np.array_equal(agents.levels.cpu().numpy(), buf.levels.cpu().numpy()[new_ids]), it
        assert buf.active.sum().item() >= N
        # terminate half the agents for the next round
        agents.step = torch.where(torch.arange(N, device="cuda") % 2 == it % 2, agents.levels[:, L_LIFETIME],
                                  torch.zeros_like(agents.step))


def test_masked_generators_match_where():
    """The level sampler's in-place masked generators (toued_level_gen_masked, toued_batch_reset_masked,
    toued_init_tables_masked) equal the reference's where(terminated, new, old) over a full new batch."""
    from toued import prng
    from toued.agents import create_agents, create_agents_into, lecun_tables, lecun_tables_into
    from toued.env import LevelGenerator
    from toued.rollout import RolloutWrapper
    N, W, mode = 13, 64, "all_shortlife"
    gen = LevelGenerator(mode)
    ro = RolloutWrapper(mode, 20, env_workers=W)
    D = ro.obs_dim
    keys_old, keys_new = prng.split(prng.PRNGKey(3, "cuda"), N), prng.split(prng.PRNGKey(4, "cuda"), N)
    mask = (torch.arange(N, device="cuda") % 3 == 1).to(torch.uint8)
    term = mask.bool()
    old_lv, new_lv = gen(keys_old), gen(keys_new)
    lv = old_lv.clone()
    gen.regenerate(keys_new, lv, mask)
    assert torch.equal(lv, torch.where(term[:, None], new_lv, old_lv))
    (_, _), st_old = ro.batch_reset(keys_old, old_lv)
    (_, _), st_new = ro.batch_reset(keys_new, lv)
    st = st_old.clone()
    ro.batch_reset_into(keys_new, lv, st, mask)
    nf = 4 + ro.spec.max_n_objs     # time, pos, exists, early_term, obj_poss[max_n_objs] (the rest is never written)
    ref = torch.where(term.repeat_interleave(W)[None, :], st_new, st_old)
    assert torch.equal(st[:nf], ref[:nf])
    th_old, ph_old = create_agents(keys_old, D, 8)
    th_new, ph_new = create_agents(keys_new, D, 8)
    th, ph = th_old.clone(), ph_old.clone()
    create_agents_into(keys_new, th, ph, mask)
    assert torch.equal(th, torch.where(term[:, None, None], th_new, th_old))
    assert torch.equal(ph, torch.where(term[:, None, None], ph_new, ph_old))
    vc = lecun_tables(keys_old, D, 1)
    vc_new = lecun_tables(keys_new, D, 1)
    lecun_tables_into(keys_new, vc, mask)
    assert torch.equal(vc, torch.where(term[:, None, None], vc_new, lecun_tables(keys_old, D, 1)))
