"""The reference-shaped Python surface on the GPU: meta/meta.py's create_lpg_train_state / make_lpg_train_step
(the functional 4-tuple step) and RolloutWrapper's single-agent call forms (environments/rollout.py:38-102)."""
import numpy as np
import pytest
import torch

from oracle import jaxrand as jr

pytestmark = pytest.mark.gpu


def test_make_lpg_train_step_matches_meta_grad_step():
    """lpg_train_step_fn(rng, lpg_train_state, agent_states, value_critic_states) -> 4-tuple (meta/meta.py:33-52,
    meta/train.py:14-130) does exactly what MetaGradStep does, and create_lpg_train_state is the flax init."""
    import toued
    from test_gpu_meta import _agents_for, _clone_agents
    from toued import prng
    from toued.level_sampler import LevelSampler
    from toued.lpg import flax_init_lpg_params
    from toued.meta import AdamState, MetaGradStep, lpg_hypers_from_args
    from toued.parse_args import parse_args
    args = parse_args(["--env_mode", "dense", "--num_agents", "4", "--num_mini_batches", "1",
                       "--num_agent_updates", "2"])
    sampler = LevelSampler(args, torch.device("cuda"))
    rng = prng.from_uint32_numpy(jr.PRNGKey(7), "cuda")
    ts = toued.create_lpg_train_state(rng, args)
    assert torch.equal(ts.params, flax_init_lpg_params(rng, 5)) and ts.step == 0
    _, ag = _agents_for("dense", 4, 64, sampler.rollout_manager.train_rollout_len, 40)
    ag2 = _clone_agents(ag)
    step = toued.make_lpg_train_step(args, sampler)
    key = prng.from_uint32_numpy(jr.PRNGKey(8), "cuda")
    vcs = toued.ValueCriticStates(ag.vcrit, ag.vstep)
    ts_out, ag_out, vc_out, m = step(key, ts, ag, vcs)
    assert ts_out.step == 1 and ag_out is ag and set(m) >= {"lpg_loss", "lpg_agent_return", "lpg_agent"}
    eta2, adam2 = flax_init_lpg_params(rng, 5), AdamState(ts.params.numel(), "cuda")
    ref = MetaGradStep(sampler.rollout_manager, 4, lpg_hypers_from_args(args, sampler), False, "cuda")
    m2 = ref(key, eta2, adam2, ag2)
    torch.cuda.synchronize()
    assert torch.equal(ts_out.params, eta2) and torch.equal(ts_out.opt.m, adam2.m)
    assert torch.equal(ag_out.theta, ag2.theta) and torch.equal(vc_out.step, ag2.vstep)
    assert torch.equal(m["lpg_loss"], m2["lpg_loss"])


def test_rollout_single_agent_forms():
    """batch_reset(rng, level, W) / batch_rollout(rng, theta[D, 5], level, state) on one agent equal the agent-axis
    call for that agent, results without the agent axis."""
    from toued.env import LevelGenerator
    from toued.prng import from_uint32_numpy
    from toued.rollout import RolloutWrapper
    dk = lambda a: from_uint32_numpy(a, "cuda")
    N, W, T = 3, 64, 17
    lev = LevelGenerator("dense")(dk(jr.split(jr.PRNGKey(1), N)))
    ro = RolloutWrapper("dense", T, env_workers=W)
    rk, ak = jr.split(jr.PRNGKey(2), N), jr.split(jr.PRNGKey(3), N)
    th = torch.from_numpy((np.random.RandomState(0).randn(N, ro.obs_dim, 5) * 2).astype(np.float32)).cuda()
    (i_all, _), st_all = ro.batch_reset(dk(rk), lev)
    tr_all, _, cum_all = ro.batch_rollout(dk(ak), th, lev, st_all)
    a = 1
    (i1, _), st1 = ro.batch_reset(dk(rk[a]), lev[a])
    f = 4 + ro.spec.max_n_objs   # state rows the env writes (time, pos, exists, early_term, object cells)
    assert torch.equal(st1[:f], st_all[:f, a * W:(a + 1) * W]) and torch.equal(i1, i_all[a * W:(a + 1) * W])
    tr1, _, cum1 = ro.batch_rollout(dk(ak[a]), th[a], lev[a], st1)
    assert tr1.action.shape == (T, W) and cum1.shape == (W,)
    assert torch.equal(tr1.action, tr_all.action[a]) and torch.equal(tr1.obs_idx, tr_all.obs_idx[a])
    assert torch.equal(cum1, cum_all[a])
