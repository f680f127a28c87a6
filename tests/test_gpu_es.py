"""GPU parity of the TA-LPG / OpenES path (meta/train.py:133-227) vs the oracles.

  * OpenES ask (normal noise, antithetic reorder, sharded rows): bit-exact vs oracle/es.py
  * OpenES tell (population dot + Adam): within 1e-5 relative of the float64 oracle
  * per-candidate LPG forward (toued_gru_fwd_multi): each candidate's rows match the float64
    oracle GRU with that candidate's parameters (same tolerance as the shared-eta forward test)
  * one ES step with K=1 agent updates: rollouts bit-exact, each candidate's updated agent within
    float32 tolerance of oracle/meta.py lpg_agent_step under its own LPG, fitness within 1e-5 of
    oracle eval_agent on the device's trained actor, pair ranks / winners consistent
"""
import numpy as np
import pytest
import torch

from oracle import agents as oag
from oracle import es as oes
from oracle import jaxrand as jr
from oracle import levels as olv
from oracle import lpg as olpg
from oracle import meta as ometa

pytestmark = pytest.mark.gpu


def dk(a):
    from toued.prng import from_uint32_numpy
    return from_uint32_numpy(a, "cuda")


@pytest.mark.parametrize("nd,pop,lo,n", [(1000, 8, 0, 4), (777, 16, 3, 4), (205482, 4, 1, 1)])
def test_es_ask_bitexact(nd, pop, lo, n):
    from toued.es import OpenES
    es = OpenES(pop, nd, sigma_init=0.1, device="cuda")
    es.mean.copy_(torch.from_numpy(np.random.RandomState(0).randn(nd).astype(np.float32)))
    key = jr.PRNGKey(nd)
    out = torch.empty(2 * n, nd, device="cuda")
    es.ask(dk(key), lo, n, out)
    ref = oes.ask(key, es.mean.cpu().numpy(), np.float32(0.1), pop)
    assert np.array_equal(out.cpu().numpy(), ref[2 * lo:2 * (lo + n)])


@pytest.mark.parametrize("opt", ["adam", "sgd"])
def test_es_tell_matches_oracle(opt):
    from toued.es import OpenES
    nd, pop = 3000, 16
    es = OpenES(pop, nd, opt_name=opt, lrate_init=0.01, lrate_decay=0.999, lrate_limit=1e-5, sigma_init=0.1,
                sigma_decay=0.99, sigma_limit=0.05, device="cuda")
    st = {"mean": np.zeros(nd), "m": np.zeros(nd), "v": np.zeros(nd), "n": 0, "lrate": 0.01, "sigma": 0.1,
          "lrate_decay": 0.999, "lrate_limit": 1e-5, "sigma_decay": 0.99, "sigma_limit": 0.05}
    rs = np.random.RandomState(1)
    x = torch.empty(pop, nd, device="cuda")
    for gen in range(3):
        es.ask(dk(jr.PRNGKey(gen)), 0, pop // 2, x)
        fit = rs.randn(pop).astype(np.float32)
        rank, _ = oes.pair_rank(fit)
        xs = x.cpu().numpy()
        st = oes.tell(xs, rank, st, opt)
        es.tell(x, torch.from_numpy(rank).cuda())
        got = es.mean.cpu().numpy()
        np.testing.assert_allclose(got, st["mean"], rtol=1e-5, atol=1e-7 * max(1.0, np.abs(st["mean"]).max()))
        st["mean"] = got.astype(np.float64)   # continue from the device state (ask uses f32 mean)
        assert abs(float(es.sigma) - st["sigma"]) < 1e-7 and abs(float(es.lrate) - st["lrate"]) < 1e-9


def test_gru_fwd_multi_per_candidate():
    from toued import _lib
    from toued.lpg import LPGLayout, init_lpg_params
    C, W, T, F = 3, 64, 20, 7
    R = C * W
    lay = LPGLayout(F)
    etas = torch.stack([init_lpg_params(10 + c, F) + torch.randn(lay.size, device="cuda") * 0.05
                        for c in range(C)]).contiguous()
    fwdA = torch.zeros(C, _lib.lib().toued_gru_packed_floats(2), device="cuda")
    _lib.call("toued_gru_pack_fwd_multi", _lib.ptr(etas), lay.size, C, lay.c_offsets, F, _lib.ptr(fwdA),
              _lib.stream_ptr())
    rs = np.random.RandomState(0)
    X = torch.from_numpy(rs.randn(F, T, R).astype(np.float32)).cuda()
    done = (rs.rand(C, T, W) < 0.1).astype(np.uint8)
    X[1] = torch.from_numpy(done.transpose(1, 0, 2).reshape(T, R).astype(np.float32)).cuda()
    pi_hat = torch.zeros(T, R, device="cuda")
    y_hat = torch.zeros(T, 8, R, device="cuda")
    _lib.call("toued_gru_fwd_multi", R, T, W, F, W, _lib.ptr(X), T * R, 1, _lib.ptr(torch.from_numpy(done).cuda()),
              _lib.ptr(fwdA), _lib.ptr(etas), lay.size, lay.c_offsets, _lib.ptr(pi_hat), _lib.ptr(y_hat),
              _lib.stream_ptr())
    torch.cuda.synchronize()
    for c in range(C):
        P = olpg.unflatten(torch.tensor(etas[c].cpu().numpy(), dtype=torch.float64), F)
        x = torch.tensor(X[:, :, c * W:(c + 1) * W].cpu().numpy(), dtype=torch.float64).permute(2, 1, 0)
        d = torch.tensor(done[c].T.astype(bool))
        h = torch.zeros(W, 256, dtype=torch.float64)
        outs = [None] * T
        for t in reversed(range(T)):
            h = torch.where(d[:, t, None], torch.zeros_like(h), h)
            xt = x[:, t]
            rg = torch.sigmoid(xt @ P["ir_w"] + P["ir_b"] + h @ P["hr_w"])
            zg = torch.sigmoid(xt @ P["iz_w"] + P["iz_b"] + h @ P["hz_w"])
            ng = torch.tanh(xt @ P["in_w"] + P["in_b"] + rg * (h @ P["hn_w"] + P["hn_b"]))
            h = (1 - zg) * ng + zg * h
            outs[t] = h
        hs = torch.relu(torch.stack(outs, 1))
        pi_ref = (hs @ P["pi_w"] + P["pi_b"])[..., 0]
        y_ref = torch.softmax(hs @ P["y_w"] + P["y_b"], -1)
        np.testing.assert_allclose(pi_hat[:, c * W:(c + 1) * W].cpu().numpy().T, pi_ref.numpy(), atol=1e-4,
                                   rtol=1e-4)
        np.testing.assert_allclose(y_hat[:, :, c * W:(c + 1) * W].cpu().numpy().transpose(2, 0, 1), y_ref.numpy(),
                                   atol=1e-5, rtol=1e-4)


def test_es_step_k1_matches_oracle():
    from toued import prng
    from toued.es import ESTrainStep
    from toued.level_sampler import LevelSampler
    from toued.parse_args import parse_args
    mode, N = "all_vrandlife", 2
    args = parse_args(["--env_mode", mode, "--num_agents", str(N), "--num_mini_batches", "1", "--use_es",
                       "--lifetime_conditioning", "--lpg_learning_rate", "0.01"])
    smp = LevelSampler(args)
    buf = smp.initialize_buffer(prng.PRNGKey(0, "cuda"))
    _, agents = smp.initial_sample(prng.PRNGKey(1, "cuda"), buf, N, False)
    agents.theta.mul_(20.0)
    agents.phi.mul_(20.0)
    from toued.lpg import LPGLayout
    eta0 = torch.zeros(LPGLayout(7).size, device="cuda")
    step = ESTrainStep(args, smp, N, eta0, "cuda", None, num_agent_updates=1)
    # non-zero search mean so the candidate LPGs produce non-trivial targets
    step.es.mean.copy_(torch.from_numpy(np.random.RandomState(5).randn(step.es.nd).astype(np.float32) * 0.05))
    th0, ph0 = agents.theta.cpu().numpy(), agents.phi.cpu().numpy()
    lev = agents.levels.cpu().numpy()
    step_np = agents.step.cpu().numpy()
    rng = jr.PRNGKey(7)
    m = step(dk(rng), agents)
    torch.cuda.synchronize()
    C, W, T, D = step.C, step.W, step.T, step.D
    x = step.x.cpu().numpy()
    ks = jr.split(rng, 2)
    tr = step.tr
    idx, tm, act = tr.obs_idx.cpu().numpy(), tr.obs_time.cpu().numpy(), tr.action.cpu().numpy()
    rew, dn = tr.reward.cpu().numpy(), tr.done.cpu().numpy()
    hyp = ometa.Hypers(lifetime_conditioning=True)
    theta_dev = step.theta[1].cpu().numpy()     # K=1: one ping-pong swap
    from oracle.levels import L_LIFETIME
    for c in range(C):
        a = c // 2
        traj = {"idx": idx[c].T.copy(), "time": tm[c].T.copy(), "action": act[c].T.astype(np.int64),
                "reward": rew[c].T.copy(), "done": dn[c].T.astype(bool)}
        eta_c = torch.tensor(x[c], dtype=torch.float64)
        th1, ph1, s1, _, _ = ometa.lpg_agent_step(torch.tensor(th0[a], dtype=torch.float64, requires_grad=True),
                                                  torch.tensor(ph0[a], dtype=torch.float64, requires_grad=True),
                                                  int(step_np[a]),
                                                  int(lev[a, L_LIFETIME]), eta_c, traj, hyp)
        d_ref = th1.detach().numpy() - th0[a]
        d_dev = theta_dev[c].astype(np.float64) - th0[a]
        assert np.linalg.norm(d_dev - d_ref) <= 2e-4 * np.linalg.norm(d_ref) + 1e-6, c
    # fitness = eval_agent(rng_c) on the device-trained actor
    ck = jr.split(jr.split(ks[0], 2)[1], 2 * N)
    fit_keys = jr.split(ck, 2)[:, 0]
    spec = olv.env_spec(mode)
    # initial_sample (random score function): levels from split(split(rng)[1], N)
    lkeys = jr.split(jr.split(jr.PRNGKey(1), 2)[1], N)
    p_lv, lt = olv.reset_env_params(lkeys, mode)
    assert np.array_equal(olv.pack_levels(p_lv, lt, spec), lev)
    p2 = {k: np.repeat(v, 2, axis=0) for k, v in p_lv.items()}
    fit_ref = oag.eval_agent(spec, fit_keys, p2, theta_dev, W, smp.max_rollout_len)
    np.testing.assert_allclose(step.fitness.cpu().numpy(), fit_ref, atol=1e-5)
    f = step.fitness.cpu().numpy()
    rank, fg = oes.pair_rank(f)
    winners = np.where(fg, np.arange(N) * 2, np.arange(N) * 2 + 1)
    assert np.array_equal(agents.theta.cpu().numpy(), theta_dev[winners])
    assert float(m["fitness"]["max"]) == pytest.approx(float(f.max()))
