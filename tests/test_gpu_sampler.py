"""GPU parity of the LPG meta-optimiser step and of LevelSampler's non-PLR branches.

  * toued_adam (optax 0.1.5 scale_by_adam + scale(lr) + scale(-1) on the agent-mean gradient,
    models/optim.py:12-17, meta/train.py:128): bit-exact vs the float32 restatement oracle/meta.adam_f32
    over several steps, and through a whole MetaGradStep (eta after the step).
  * LevelSampler.initial_sample / sample for score_function random and frozen
    (level_sampler.py:90-167, 237-291): levels, env states, actor/critic/value-critic tables and
    steps bit-exact vs oracle/sampler.py, including which agents are regenerated (terminated mask).
  * initial_sample for the buffer score functions (alg_regret): the agents' keys (no split before the
    agents outside the random branch, level_sampler.py:112-119).
"""
import numpy as np
import pytest
import torch

from oracle import jaxrand as jr
from oracle import levels as olv
from oracle import meta as ometa
from oracle import sampler as osp

pytestmark = pytest.mark.gpu


def dk(a):
    from toued.prng import from_uint32_numpy
    return from_uint32_numpy(a, "cuda")


def test_adam_bitexact_multi_step():
    from toued import _lib
    P, n = 100_003, 7
    rs = np.random.RandomState(0)
    eta = rs.randn(P).astype(np.float32) * 0.1
    m = np.zeros(P, np.float32)
    v = np.zeros(P, np.float32)
    d_eta, d_m, d_v = (torch.from_numpy(x.copy()).cuda() for x in (eta, m, v))
    count = 0
    for it in range(4):
        g = (rs.randn(P) * 10.0 ** rs.randint(-6, 3, P)).astype(np.float32)
        g[:5] = [0.0, -0.0, 1e-30, 3e4, -7.5]
        d_g = torch.from_numpy(g).cuda()
        _lib.call("toued_adam", P, _lib.ptr(d_eta), _lib.ptr(d_g), _lib.ptr(d_m), _lib.ptr(d_v), float(n), 1e-4, 0.9,
                  0.999, 1e-8, count + 1, _lib.stream_ptr())
        eta, m, v, count = ometa.adam_f32(eta, g, n, m, v, count)
        torch.cuda.synchronize()
        assert np.array_equal(d_m.cpu().numpy(), m), it
        assert np.array_equal(d_v.cpu().numpy(), v), it
        assert np.array_equal(d_eta.cpu().numpy(), eta), it


def test_adam_inside_meta_step():
    """eta after MetaGradStep == adam_f32(eta_before, the step's summed meta-gradient, N): the Adam link of
    lpg_meta_grad_train_step (meta/train.py:127-129) on the real gradient."""
    from test_gpu_meta import _setup
    N = 2
    agents, step, eta, adam, hyp, D = _setup("dense", N, 64, 20, 2)
    eta0 = eta.cpu().numpy()
    step(torch.tensor([0, 9], dtype=torch.int32, device="cuda"), eta, adam, agents)
    torch.cuda.synchronize()
    ref, m, v, c = ometa.adam_f32(eta0, step.grad.cpu().numpy(), N, np.zeros_like(eta0), np.zeros_like(eta0), 0)
    assert adam.count == c == 1
    assert np.array_equal(eta.cpu().numpy(), ref)
    assert np.array_equal(adam.m.cpu().numpy(), m)
    assert np.array_equal(adam.v.cpu().numpy(), v)


def _check_agents(spec, agents, lv, th, ph, st, vc, step):
    from test_gpu_env import _state_np
    np.testing.assert_array_equal(agents.levels.cpu().numpy(), olv.pack_levels(lv[0], lv[1], spec, lv[2]))
    np.testing.assert_array_equal(agents.theta.cpu().numpy(), th)
    np.testing.assert_array_equal(agents.phi.cpu().numpy(), ph)
    g = _state_np(agents.state, spec)
    for k in ("time", "pos", "obj_existss", "early_term", "obj_poss"):
        np.testing.assert_array_equal(g[k], st[k], err_msg=k)
    if vc is not None:
        np.testing.assert_array_equal(agents.vcrit.cpu().numpy().reshape(vc.shape), vc)
    np.testing.assert_array_equal(agents.step.cpu().numpy(), step)


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("score_function,mode", [("random", "all_shortlife"), ("frozen", "all_shortlife"),
                                                 ("random", "tabular"), ("frozen", "mazes")])
def test_sample_nonplr_matches_oracle(monkeypatch, score_function, mode, fused):
    """sample() against the oracle; the random branch both as toued_sample_random_keys + the masked generators
    (TOUED_SAMPLE_FUSED=1, default) and launch per operation (0)."""
    if fused == "0" and score_function != "random":
        pytest.skip("the flag only selects the random branch's path")
    monkeypatch.setenv("TOUED_SAMPLE_FUSED", fused)
    from toued import prng
    from toued.env import L_LIFETIME
    from toued.level_sampler import LevelSampler
    from toued.parse_args import parse_args
    N, B, W, Y = 6, 40, 64, 8
    args = parse_args(["--env_mode", mode, "--score_function", score_function, "--num_agents", str(N),
                       "--num_mini_batches", "1", "--buffer_size", str(B)])
    smp = LevelSampler(args)
    spec = olv.env_spec(mode)
    k_buf, k_init, k_s1, k_s2 = jr.split(jr.PRNGKey(51), 4)
    buf = smp.initialize_buffer(dk(k_buf))
    obuf = None
    if score_function != "random":
        obuf, _, _, _ = osp.initialize_buffer(k_buf, mode, B)
        np.testing.assert_array_equal(buf.levels.cpu().numpy(), olv.pack_levels(obuf[0], obuf[1], spec, obuf[2]))
    buf, agents = smp.initial_sample(dk(k_init), buf, N, True)
    lv, th, ph, st, vc = osp.initial_sample(spec, mode, score_function, k_init, obuf, N, W, Y, True)
    step = np.zeros(N, np.int32)
    _check_agents(spec, agents, lv, th, ph, st, vc, step)
    # two sample() rounds: first agents 1, 3, 4 terminated, then all but agent 0
    for key, term_ids in ((k_s1, [1, 3, 4]), (k_s2, [1, 2, 3, 4, 5])):
        term = np.zeros(N, bool)
        term[term_ids] = True
        life = agents.levels[:, L_LIFETIME].cpu().numpy()
        step = np.where(term, life, np.minimum(life - 1, 3)).astype(np.int32)
        agents.step = torch.from_numpy(step).cuda()
        # make the survivors' tables distinguishable from fresh ones
        agents.theta.add_(0.5)
        th, ph, vc = agents.theta.cpu().numpy(), agents.phi.cpu().numpy(), agents.vcrit.cpu().numpy().reshape(vc.shape)
        buf, agents = smp.sample(dk(key), buf, agents)
        lv, th, ph, st, vc, step = osp.sample_nonplr(spec, mode, score_function, key, obuf, term,
                                                     (lv, th, ph, st, vc, step), W, Y)
        torch.cuda.synchronize()
        _check_agents(spec, agents, lv, th, ph, st, vc, step)


def test_initial_sample_buffer_mode_agent_keys():
    from toued.level_sampler import LevelSampler
    from toued.parse_args import parse_args
    mode, N, B = "all_shortlife", 5, 32
    args = parse_args(["--env_mode", mode, "--score_function", "alg_regret", "--num_agents", str(N),
                       "--num_mini_batches", "1", "--buffer_size", str(B)])
    smp = LevelSampler(args)
    spec = olv.env_spec(mode)
    k_buf, k_init = jr.split(jr.PRNGKey(61), 2)
    buf = smp.initialize_buffer(dk(k_buf))
    buf, agents = smp.initial_sample(dk(k_init), buf, N, False)
    obuf, _, _, _ = osp.initialize_buffer(k_buf, mode, B)
    lv, th, ph, st, _ = osp.initial_sample(spec, mode, "alg_regret", k_init, obuf, N, 64, 8, False)
    _check_agents(spec, agents, lv, th, ph, st, None, np.zeros(N, np.int32))
    assert buf.active.cpu().numpy().tolist() == [True] * N + [False] * (B - N)


@pytest.mark.parametrize("F", [5, 7])
def test_flax_lpg_init_matches_oracle(F):
    """create_lpg_train_state (meta/meta.py:21-22): the device's flax init of eta from lpg_rng vs
    oracle/flaxinit.lpg_init — lecun_normal kernels bit-exact, orthogonal recurrent kernels within 1e-6
    (float64 QR of bit-exact normal draws on both sides), zero biases; and Trainer starts from it."""
    from oracle import flaxinit
    from toued.lpg import LPGLayout, flax_init_lpg_params
    key = jr.split(jr.PRNGKey(0), 3)[1]                       # train.py:17 rng, lpg_rng, buffer_rng
    got = flax_init_lpg_params(dk(key), F).cpu().numpy()
    ref = flaxinit.lpg_init(key, F)
    lay = LPGLayout(F)
    for name, shape in lay.shapes.items():
        o = lay.offsets[name]
        g, r = got[o:o + int(np.prod(shape))], ref[o:o + int(np.prod(shape))]
        if name in ("hn_w", "hr_w", "hz_w"):
            np.testing.assert_allclose(g, r, atol=1e-6, rtol=0, err_msg=name)
            q = g.reshape(shape).astype(np.float64)
            np.testing.assert_allclose(q.T @ q, np.eye(shape[0]), atol=1e-5)
        else:
            assert np.array_equal(g, r), name
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = ["--env_mode", "dense", "--num_agents", "2", "--num_mini_batches", "1"]
    if F == 7:
        args.append("--lifetime_conditioning")
    tr = Trainer(parse_args(args))
    assert np.array_equal(tr.eta.cpu().numpy(), got)


@pytest.mark.parametrize("fused", ["1", "0"])
def test_sample_random_rank_slice_matches_full_batch(monkeypatch, fused):
    """sample() of one rank's agent slice (sl = (lo, hi, n_total), as each rank runs it under data parallelism) equals
    that slice of the full-batch sample: levels, tables, value critics, env states and step counters, with agents
    terminated on both sides of the slice; the random branch as toued_sample_random_keys (1) and launch per
    operation (0)."""
    monkeypatch.setenv("TOUED_SAMPLE_FUSED", fused)
    from toued.agents import AgentBatch
    from toued.env import L_LIFETIME
    from toued.level_sampler import LevelSampler
    from toued.parse_args import parse_args
    N, W, lo, hi = 8, 64, 3, 7
    args = parse_args(["--env_mode", "all_shortlife", "--score_function", "random", "--num_agents", str(N),
                       "--num_mini_batches", "1"])
    smp = LevelSampler(args)
    k_init, k_s = jr.split(jr.PRNGKey(77), 2)
    _, full = smp.initial_sample(dk(k_init), None, N, True)
    life = full.levels[:, L_LIFETIME]
    term = torch.tensor([1, 0, 1, 1, 0, 1, 0, 1], dtype=torch.bool, device="cuda")
    full.step = torch.where(term, life, torch.ones_like(life)).to(torch.int32)
    full.vstep = full.step.clone()
    full.theta.add_(0.5)
    part = AgentBatch(full.levels[lo:hi].clone(), full.theta[lo:hi].clone(), full.phi[lo:hi].clone(),
                      full.step[lo:hi].clone(), full.state[:, lo * W:hi * W].clone(), full.vcrit[lo:hi].clone(),
                      full.vstep[lo:hi].clone())
    _, full = smp.sample(dk(k_s), None, full)
    _, part = smp.sample(dk(k_s), None, part, (lo, hi, N))
    torch.cuda.synchronize()
    assert torch.equal(part.levels, full.levels[lo:hi])
    assert torch.equal(part.theta, full.theta[lo:hi]) and torch.equal(part.phi, full.phi[lo:hi])
    assert torch.equal(part.vcrit, full.vcrit[lo:hi])
    assert torch.equal(part.step, full.step[lo:hi]) and torch.equal(part.vstep, full.vstep[lo:hi])
    assert torch.equal(part.state, full.state[:, lo * W:hi * W])
    assert bool((full.step[term] == 0).all()) and bool((full.step[~term] == 1).all())   # only terminated ones reset
