"""GPU parity of the TA-LPG / OpenES path (meta/train.py:133-227) vs the oracles.

  * OpenES ask (normal noise, antithetic reorder, sharded rows): bit-exact vs oracle/es.py
  * OpenES tell (population dot + Adam): within 1e-5 relative of the float64 oracle
  * per-candidate LPG forward (toued_gru_fwd_multi): each candidate's rows match the float64
    oracle GRU with that candidate's parameters within 5e-6 absolute (the shared-eta forward's bound)
  * one ES step with K=1 agent update: each candidate's updated agent (on the device's trajectory) within
    float32 tolerance of oracle/meta.py lpg_agent_step under its own LPG, fitness within 1e-5 of oracle
    eval_agent on the device's trained actor, pair ranks / winners consistent
  * one ES step with K=3 agent updates (test_es_step_k3_matches_oracle): ask bit-exact, every candidate's
    K rollouts regenerated bit-exactly by oracle/rollout.py from the oracle's own key chain
    (meta/train.py:160-200, lpg_agent.py:107) and the device's theta_k, each agent update and the K chained
    float64 agent updates within 2e-5, the agent metrics within 2e-5, fitness within 1e-5, and the in-step rank -> tell: the
    population gradient within 1e-6 relative L2, the Adam step on it within f32 rounding (meta/train.py:203-217)
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
from oracle import rollout as oro

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
    gen = torch.Generator(device="cuda").manual_seed(1234)   # seeded: the same inputs on every run
    etas = torch.stack([init_lpg_params(10 + c, F) + torch.randn(lay.size, device="cuda", generator=gen) * 0.05
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
        np.testing.assert_allclose(pi_hat[:, c * W:(c + 1) * W].cpu().numpy().T, pi_ref.numpy(), atol=5e-6, rtol=0)
        np.testing.assert_allclose(y_hat[:, :, c * W:(c + 1) * W].cpu().numpy().transpose(2, 0, 1), y_ref.numpy(),
                                   atol=5e-6, rtol=0)


def test_track_best_on_device_matches_evosax_rule():
    """OpenES.track_best (device-side, no host sync) against evosax 0.1.4's get_best_fitness_member restated on the
    host: first index of the largest fitness, replaced only when it beats the stored best in the minimisation frame
    (gen 0 compares against the raw initial value), over generations with ties, a worse generation and a slice of
    the population held locally (lo > 0)."""
    from toued.es import OpenES
    nd, pop = 37, 8
    es = OpenES(pop, nd, device="cuda")
    rs = np.random.RandomState(3)
    x = torch.from_numpy(rs.randn(pop, nd).astype(np.float32)).cuda()
    host_best, host_member = np.float32(np.finfo(np.float32).max), None
    fits = [np.array([0.2, 0.9, 0.9, 0.1, 0.0, 0.5, 0.3, 0.9], np.float32),      # ties: the first maximum
            np.array([0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8], np.float32),      # worse: no replacement
            np.array([0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.95, 0.0], np.float32)]     # better, in the slice below
    lo = 2
    for g, fit in enumerate(fits):
        fmin = -fit
        i = int(np.argmin(fmin))
        best_min = -host_best if g > 0 else host_best
        if fmin[i] < best_min:
            host_member = x[i].cpu().numpy().copy()
            best_min = fmin[i]
        host_best = np.float32(-best_min)
        es.track_best(x[lo:], torch.from_numpy(fit).cuda(), lo) if g == 2 else es.track_best(x, torch.from_numpy(fit).cuda(), 0)
        es.gen_counter += 1
        assert es.best_fitness == host_best, g
        np.testing.assert_array_equal(es.best_member.cpu().numpy(), host_member, err_msg=str(g))


def test_es_fused_agent_update_bitexact():
    """toued_agent_update (gradient + clip + SGD in place, the ES default) against toued_agent_grad + toued_agent_apply
    into ping-pong tables: three agent updates per candidate, lifetime 2 on one agent (a discarded update), the ES
    step's outputs bit-identical -- winners' tables, steps, env state, metrics, fitness and the new search mean."""
    from toued import prng
    from toued.env import L_LIFETIME
    from toued.es import ESTrainStep
    from toued.level_sampler import LevelSampler
    from toued.lpg import LPGLayout
    from toued.parse_args import parse_args
    mode, N = "all_vrandlife", 3
    args = parse_args(["--env_mode", mode, "--num_agents", str(N), "--num_mini_batches", "1", "--use_es",
                       "--lifetime_conditioning", "--lpg_learning_rate", "0.01"])
    outs = []
    for fused in (False, True):
        smp = LevelSampler(args)
        buf = smp.initialize_buffer(prng.PRNGKey(0, "cuda"))
        _, agents = smp.initial_sample(prng.PRNGKey(1, "cuda"), buf, N, False)
        agents.theta.mul_(20.0)
        agents.phi.mul_(20.0)
        agents.levels[1, L_LIFETIME] = 2
        step = ESTrainStep(args, smp, N, torch.zeros(LPGLayout(7).size, device="cuda"), "cuda", None,
                           num_agent_updates=3)
        assert step.fused_update                      # the default where the sizes fit
        step.fused_update = fused
        step.es.mean.copy_(torch.from_numpy(np.random.RandomState(5).randn(step.es.nd).astype(np.float32) * 0.05))
        m = step(dk(jr.PRNGKey(7)), agents)
        torch.cuda.synchronize()
        outs.append((agents.theta.clone(), agents.phi.clone(), agents.step.clone(), agents.state.clone(),
                     step.fitness.clone(), step.es.mean.clone(), step.gstat.clone(),
                     {k: torch.as_tensor(v).detach().clone() for k, v in _flat(m).items()}))
    nrow = 4 + olv.env_spec(mode).max_n_objs      # state rows the env uses (the rest are never written)
    # gstat of the last update: norms and the applied flag (step + 1 <= lifetime, read before the step advances)
    for i, name in enumerate(("theta", "phi", "step", "state", "fitness", "es mean", "gstat")):
        a, b = (outs[0][i][:nrow], outs[1][i][:nrow]) if name == "state" else (outs[0][i], outs[1][i])
        assert torch.equal(a, b), name
    assert outs[0][7].keys() == outs[1][7].keys()
    for k in outs[0][7]:
        assert torch.equal(outs[0][7][k], outs[1][7][k]), k


def _flat(m, pre=""):
    out = {}
    for k, v in m.items():
        if isinstance(v, dict):
            out.update(_flat(v, pre + k + "."))
        else:
            out[pre + k] = v
    return out


def test_es_step_k1_matches_oracle():
    """K = 1: the device's one trajectory per candidate is fed to the oracle update (the K = 3 test below also
    regenerates the rollouts)."""
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
    theta_dev = step.theta[step.cur].cpu().numpy()     # the candidates' tables after the update
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
        assert np.linalg.norm(d_dev - d_ref) <= 2e-5 * np.linalg.norm(d_ref) + 1e-7, c
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


def certify_es_step(args, smp, step, rng, pre, metrics, p_lv, chained=False):
    """Every stage of one lpg_es_train_step (meta/train.py:133-227) against the oracle, from the device state
    before it (pre: es mean/m/v/n/lrate/sigma, the agents' theta/phi/step/env state/packed levels; p_lv: the
    oracle's EnvParams of those levels, checked against the packed ones) and the
    step's trace (ESTrainStep.trace): ask bit-exact; every candidate's K rollouts regenerated bit-exactly from
    the oracle's own key chain (:160-200, lpg_agent.py:107) and the device's theta_k; each of the K agent updates
    (from the device's tables before it) within 2e-5 relative L2 of the float64 update under the candidate's LPG,
    and the agent metrics within 2e-5; fitness = eval_agent within 1e-5;
    winners; the rank -> tell -> mean within 1e-5 of oracle/es.tell.  Returns (fitness, oracle fitness)."""
    from test_gpu_env import _state_np
    from oracle.levels import L_LIFETIME
    mode = args.env_mode
    N, C, W, T, K = step.N, step.C, step.W, step.T, step.K
    assert len(step.trace) == K
    x = step.x.cpu().numpy()
    lev = pre["levels"]
    r1, sub = jr.split(rng, 2)
    np.testing.assert_array_equal(x, oes.ask(sub, pre["mean"], np.float32(pre["sigma"]), C))
    _, sub2 = jr.split(r1, 2)
    ck2 = jr.split(jr.split(sub2, C), 2)
    fit_keys, tk = ck2[:, 0], ck2[:, 1]
    spec = olv.env_spec(mode)
    p2 = {kk: np.repeat(v, 2, axis=0) for kk, v in p_lv.items()}
    st_rep = torch.from_numpy(pre["state"]).view(12, N, W).repeat_interleave(2, dim=1).reshape(12, C * W)
    ost = _state_np(st_rep, spec)
    trajs = []
    for k in range(K):
        s2 = jr.split(tk, 2)
        tk, rk = s2[:, 0], s2[:, 1]
        th_k = step.trace[k]["theta"].cpu().numpy()
        otr, ost, _ = oro.batch_rollout(spec, rk, th_k, p2, ost, T)
        tr = step.trace[k]["traj"]
        for name, got in (("idx", tr.obs_idx), ("time", tr.obs_time), ("action", tr.action), ("reward", tr.reward),
                          ("done", tr.done)):
            g = got.cpu().numpy()
            np.testing.assert_array_equal(g, otr[name].transpose(0, 2, 1).astype(g.dtype), err_msg=f"rollout {k} {name}")
        trajs.append({"idx": otr["idx"], "time": otr["time"], "action": otr["action"].astype(np.int64),
                      "reward": otr["reward"], "done": otr["done"].astype(bool)})
    hyp = ometa.Hypers(lifetime_conditioning=step.F == 7)
    th_dev, ph_dev = step.theta[step.cur].cpu().numpy(), step.phi[step.cur].cpu().numpy()
    # every update from the device's tables before it (trace): the parameter change within 2e-5 relative L2 of the
    # float64 update under the candidate's LPG (per update, as _a2c_follow: chained over K updates at the actor
    # lr 40 the float32 rounding of one update is amplified into the next one's inputs)
    th_k = [r["theta"].cpu().numpy() for r in step.trace] + [th_dev]
    ph_k = [r["phi"].cpu().numpy() for r in step.trace] + [ph_dev]
    st_k = [r["step"].cpu().numpy() for r in step.trace]
    steps_ref = []
    for c in range(C):
        a = c // 2
        eta_c = torch.tensor(x[c], dtype=torch.float64)
        s = int(pre["step"][a])
        mets = []
        for k in range(K):
            assert int(st_k[k][c]) == s, (c, k)
            tr_c = {kk: v[c] for kk, v in trajs[k].items()}
            th = torch.tensor(th_k[k][c], dtype=torch.float64, requires_grad=True)
            ph = torch.tensor(ph_k[k][c], dtype=torch.float64, requires_grad=True)
            th1, ph1, s, mk, _ = ometa.lpg_agent_step(th, ph, s, int(lev[a, L_LIFETIME]), eta_c, tr_c, hyp)
            for got0, got1, ref1, nm in ((th_k[k][c], th_k[k + 1][c], th1, "theta"), (ph_k[k][c], ph_k[k + 1][c], ph1, "phi")):
                d_ref = ref1.detach().numpy() - got0
                d_dev = got1.astype(np.float64) - got0
                assert np.linalg.norm(d_dev - d_ref) <= 2e-5 * np.linalg.norm(d_ref) + 1e-7, (nm, c, k)
            t1 = torch.tensor(th_k[k + 1][c], dtype=torch.float64)
            p1 = torch.tensor(ph_k[k + 1][c], dtype=torch.float64)
            pe = ometa.entropy(torch.softmax(ometa.linear_logits(t1, tr_c["idx"][:, :-1], tr_c["time"][:, :-1]), -1))
            ce = ometa.entropy(torch.softmax(ometa.linear_logits(p1, tr_c["idx"][:, :-1], tr_c["time"][:, :-1]), -1))
            mets.append({**{kk: float(v) for kk, v in mk.items()}, "policy_entropy": float(pe),
                         "critic_entropy": float(ce)})
        steps_ref.append(s)
        if chained:   # and the K updates chained in float64 from the tables before the step, within 2e-5
            th = torch.tensor(pre["theta"][a], dtype=torch.float64, requires_grad=True)
            ph = torch.tensor(pre["phi"][a], dtype=torch.float64, requires_grad=True)
            s2 = int(pre["step"][a])
            for k in range(K):
                tr_c = {kk: v[c] for kk, v in trajs[k].items()}
                th, ph, s2, _, _ = ometa.lpg_agent_step(th, ph, s2, int(lev[a, L_LIFETIME]), eta_c, tr_c, hyp)
                th, ph = th.detach().requires_grad_(), ph.detach().requires_grad_()
            np.testing.assert_allclose(th_dev[c], th.detach().numpy(), rtol=2e-5, atol=2e-5, err_msg=f"theta {c}")
            np.testing.assert_allclose(ph_dev[c], ph.detach().numpy(), rtol=2e-5, atol=2e-5, err_msg=f"phi {c}")
        for key in ("critic_loss", "policy_l2", "critic_l2", "policy_entropy", "critic_entropy"):
            ref = np.mean([mm[key] for mm in mets])
            np.testing.assert_allclose(float(metrics["lpg_agent"][key][c]), ref, rtol=2e-5, atol=1e-7, err_msg=key)
    fit_ref = oag.eval_agent(spec, fit_keys, p2, th_dev, W, step.sampler.max_rollout_len)
    f = step.fitness.cpu().numpy()
    np.testing.assert_allclose(f, fit_ref, atol=1e-5)
    rank, fg = oes.pair_rank(f)
    winners = np.where(fg, np.arange(N) * 2, np.arange(N) * 2 + 1)
    assert float(metrics["fitness"]["mean"]) == pytest.approx(float(f.mean()), rel=1e-6, abs=1e-9)
    st = {"mean": pre["mean"].astype(np.float64), "m": pre["m"].astype(np.float64), "v": pre["v"].astype(np.float64),
          "n": pre["n"], "lrate": pre["lrate"], "sigma": pre["sigma"], "lrate_decay": args.es_lrate_decay,
          "lrate_limit": args.es_lrate_limit, "sigma_decay": args.es_sigma_decay, "sigma_limit": args.es_sigma_limit}
    # the population gradient within 1e-6 relative L2 of float64 (the device's per-parameter f32 dot over the
    # candidates), then the optimiser step from the device's gradient within f32 rounding.  (Adam divides by
    # sqrt(v): where the few antithetic terms of a parameter's dot cancel, |g| approaches eps and the update's
    # value depends on the gradient's last bits -- compared end to end it is ill-conditioned at such elements.)
    g_ref = oes.grad(x, rank, st)
    g_dev = step.es.grad.cpu().numpy().astype(np.float64) / (step.es.popsize * pre["sigma"])
    assert np.linalg.norm(g_dev - g_ref) <= 1e-6 * np.linalg.norm(g_ref), np.linalg.norm(g_dev - g_ref)
    st = oes.opt_step(g_dev, st, args.lpg_opt.lower())
    got = step.es.mean.cpu().numpy()
    np.testing.assert_allclose(got, st["mean"], rtol=1e-6, atol=2e-8)   # atol: a few f32 ulps of O(0.1) operands
    assert float(step.es.sigma) == pytest.approx(st["sigma"], abs=1e-7)
    return f, fit_ref, winners, np.array(steps_ref)[winners], th_dev[winners], ph_dev[winners], ost


def es_pre(step, agents):
    es = step.es
    return {"mean": es.mean.cpu().numpy(), "m": es.m.cpu().numpy(), "v": es.v.cpu().numpy(), "n": es.n,
            "lrate": float(es.lrate), "sigma": float(es.sigma), "theta": agents.theta.cpu().numpy(),
            "phi": agents.phi.cpu().numpy(), "step": agents.step.cpu().numpy(), "state": agents.state.cpu().numpy(),
            "levels": agents.levels.cpu().numpy()}


def test_es_step_k3_matches_oracle():
    """lpg_es_train_step (meta/train.py:133-227) with K = 3 agent updates per candidate at N = 2 (4 candidates),
    all_vrandlife with lifetime conditioning, every stage against the oracle from the oracle's own key chain
    (certify_es_step); the kept agents are the pair winners' trained tables."""
    from toued import prng
    from toued.es import ESTrainStep
    from toued.level_sampler import LevelSampler
    from toued.lpg import LPGLayout
    from toued.parse_args import parse_args
    mode, N, K = "all_vrandlife", 2, 3
    args = parse_args(["--env_mode", mode, "--num_agents", str(N), "--num_mini_batches", "1", "--use_es",
                       "--lifetime_conditioning", "--lpg_learning_rate", "0.01"])
    smp = LevelSampler(args)
    buf = smp.initialize_buffer(prng.PRNGKey(0, "cuda"))
    _, agents = smp.initial_sample(prng.PRNGKey(1, "cuda"), buf, N, False)
    agents.theta.mul_(20.0)
    agents.phi.mul_(20.0)
    step = ESTrainStep(args, smp, N, torch.zeros(LPGLayout(7).size, device="cuda"), "cuda", None,
                       num_agent_updates=K)
    step.es.mean.copy_(torch.from_numpy(np.random.RandomState(5).randn(step.es.nd).astype(np.float32) * 0.05))
    pre = es_pre(step, agents)
    spec = olv.env_spec(mode)
    p_lv, lt = olv.reset_env_params(jr.split(jr.split(jr.PRNGKey(1), 2)[1], N), mode)
    assert np.array_equal(olv.pack_levels(p_lv, lt, spec), pre["levels"])
    step.trace = []
    rng = jr.PRNGKey(11)
    m = step(dk(rng), agents)
    torch.cuda.synchronize()
    _, _, winners, steps_w, th_w, ph_w, _ = certify_es_step(args, smp, step, rng, pre, m, p_lv, chained=True)
    assert np.array_equal(agents.theta.cpu().numpy(), th_w) and np.array_equal(agents.phi.cpu().numpy(), ph_w)
    assert np.array_equal(agents.step.cpu().numpy(), steps_w)


def test_es_draws_ahead_bit_identical(monkeypatch):
    """The ES step with its rollout draws made one chunk ahead on a side stream (double-buffered, three chunks at
    K = 70) and the fitness eval's draws behind the last chunk's (TOUED_ES_AHEAD=1, an option: measured no faster)
    is bit-identical to the in-order default (TOUED_ES_AHEAD=0): fitness, kept agents, env states and the ES
    state."""
    from toued import prng
    from toued.es import ESTrainStep
    from toued.level_sampler import LevelSampler
    from toued.lpg import LPGLayout
    from toued.parse_args import parse_args
    mode, N, K = "all_vrandlife", 4, 70
    args = parse_args(["--env_mode", mode, "--num_agents", str(N), "--num_mini_batches", "1", "--use_es",
                       "--lifetime_conditioning", "--lpg_learning_rate", "0.01"])
    smp = LevelSampler(args)
    out = []
    for ahead in ("1", "0"):
        monkeypatch.setenv("TOUED_ES_AHEAD", ahead)
        buf = smp.initialize_buffer(prng.PRNGKey(0, "cuda"))
        _, agents = smp.initial_sample(prng.PRNGKey(1, "cuda"), buf, N, False)
        agents.theta.mul_(20.0)
        agents.phi.mul_(20.0)
        step = ESTrainStep(args, smp, N, torch.zeros(LPGLayout(7).size, device="cuda"), "cuda", None,
                           num_agent_updates=K)
        step.es.mean.copy_(torch.from_numpy(np.random.RandomState(5).randn(step.es.nd).astype(np.float32) * 0.05))
        step(dk(jr.PRNGKey(11)), agents)
        torch.cuda.synchronize()
        out.append([step.fitness.clone(), agents.theta.clone(), agents.phi.clone(), agents.step.clone(),
                    agents.state.clone(), step.es.mean.clone(), step.es.m.clone()])
    for a, b in zip(*out):
        assert torch.equal(a, b)
