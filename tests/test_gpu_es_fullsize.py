"""C4 (TA-LPG, --use_es) at its production size: 512 agents -> 1024 OpenES candidates, W = 64,
T = 20, F = 7 -- the bench's shape (bench.py workload_c4).  The other ES tests run at most 4 candidates, so a
candidate-index or fragment-offset slip past candidate 255 (the first round of 256 workgroups) would pass them.

  * test_gru_fwd_multi_production_size: toued_gru_fwd_multi over 1024 candidates x 64 rows x 20 steps (4 rounds of
    the 256 CUs), every candidate with its own LPG parameters; candidates {0, 1, 255, 256, 511, 767, 1022, 1023}
    against the float64 GRU + heads at the forward's 5e-6 absolute bound (meta/train.py:167-200, models/lpg.py:11-96).
  * test_es_step_production_size: one lpg_es_train_step (meta/train.py:133-227) at N = 512 on all_vrandlife with
    lifetime conditioning and K = 2 agent updates per candidate, checked by properties of the whole population and
    by the oracle on sampled candidates:
      - every fitness finite; the pair ranks and winners consistent with the fitness, and the kept agents the
        winners' trained tables, steps and env states;
      - the OpenES tell gradient against float64 noise^T (-rank) / (P sigma) of the device's own population and
        fitness (1e-6 relative L2), and the new search mean from it within f32 rounding;
      - for the sampled candidates: both rollouts regenerated bit-exactly by oracle/rollout.py from the oracle's own
        key chain (split(split(rng)[1], P) per candidate, lpg_agent.py:107) and the device's tables, each agent
        update within 2e-5 relative L2 of the float64 update under that candidate's LPG, and the fitness
        (eval_agent over 64 workers) within 1e-5 of oracle/agents.py on the device's trained tables.
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

SAMPLED = (0, 1, 255, 256, 511, 767, 1022, 1023)


def _gru_ref(P, x, d):
    """float64 reverse-time GRU + heads of one candidate (models/lpg.py:11-96): x [W, T, F], d [W, T] bool."""
    W, T = x.shape[0], x.shape[1]
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
    return (hs @ P["pi_w"] + P["pi_b"])[..., 0], torch.softmax(hs @ P["y_w"] + P["y_b"], -1)


def test_gru_fwd_multi_production_size():
    from toued import _lib
    from toued.lpg import LPGLayout, init_lpg_params
    C, W, T, F = 1024, 64, 20, 7
    R = C * W
    lay = LPGLayout(F)
    gen = torch.Generator(device="cuda").manual_seed(4321)
    base = init_lpg_params(3, F)
    # every candidate its own parameters (a perturbation of the size of the recurrent weights' entries, so that a
    # candidate computed with a neighbour's fragments or scales is off by O(0.1))
    etas = (base[None, :] + torch.randn(C, lay.size, device="cuda", generator=gen) * 0.05).contiguous()
    fwdA = torch.zeros(C, _lib.lib().toued_gru_packed_floats(2), device="cuda")
    _lib.call("toued_gru_pack_fwd_multi", _lib.ptr(etas), lay.size, C, lay.c_offsets, F, _lib.ptr(fwdA),
              _lib.stream_ptr())
    X = torch.randn(F, T, R, device="cuda", generator=gen)
    done = (torch.rand(C, T, W, device="cuda", generator=gen) < 0.1).to(torch.uint8)
    X[1] = done.permute(1, 0, 2).reshape(T, R).float()
    pi_hat = torch.full((T, R), float("nan"), device="cuda")
    y_hat = torch.full((T, 8, R), float("nan"), device="cuda")
    _lib.call("toued_gru_fwd_multi", R, T, W, F, W, _lib.ptr(X), T * R, 1, _lib.ptr(done), _lib.ptr(fwdA),
              _lib.ptr(etas), lay.size, lay.c_offsets, _lib.ptr(pi_hat), _lib.ptr(y_hat), _lib.stream_ptr())
    torch.cuda.synchronize()
    # every output written (the NaN fill would survive a skipped workgroup)
    assert bool(torch.isfinite(pi_hat).all()) and bool(torch.isfinite(y_hat).all())
    for c in SAMPLED:
        P = olpg.unflatten(etas[c].double().cpu(), F)
        x = X[:, :, c * W:(c + 1) * W].double().cpu().permute(2, 1, 0)
        d = done[c].cpu().T.bool()
        pi_ref, y_ref = _gru_ref(P, x, d)
        err_pi = float((pi_hat[:, c * W:(c + 1) * W].cpu().double().T - pi_ref).abs().max())
        err_y = float((y_hat[:, :, c * W:(c + 1) * W].cpu().double().permute(2, 0, 1) - y_ref).abs().max())
        assert err_pi <= 5e-6 and err_y <= 5e-6, (c, err_pi, err_y)


def test_es_step_production_size():
    from test_gpu_env import _state_np
    from toued import prng
    from toued.es import ESTrainStep
    from toued.level_sampler import LevelSampler
    from toued.lpg import LPGLayout
    from toued.parse_args import parse_args
    from oracle.levels import L_LIFETIME
    mode, N, K = "all_vrandlife", 512, 2
    args = parse_args(["--env_mode", mode, "--num_agents", str(N), "--num_mini_batches", "1", "--use_es",
                       "--lifetime_conditioning", "--lpg_learning_rate", "0.01"])
    smp = LevelSampler(args)
    buf = smp.initialize_buffer(prng.PRNGKey(0, "cuda"))
    _, agents = smp.initial_sample(prng.PRNGKey(1, "cuda"), buf, N, False)
    agents.theta.mul_(20.0)
    agents.phi.mul_(20.0)
    step = ESTrainStep(args, smp, N, torch.zeros(LPGLayout(7).size, device="cuda"), "cuda", None,
                       num_agent_updates=K)
    C, W, T = step.C, step.W, step.T
    assert C == 1024 and W == 64 and T == 20
    step.es.mean.copy_(torch.from_numpy(np.random.RandomState(5).randn(step.es.nd).astype(np.float32) * 0.05))
    es = step.es
    pre_mean, pre_m, pre_v, pre_n = es.mean.clone(), es.m.cpu().numpy(), es.v.cpu().numpy(), es.n
    pre_sigma, pre_lrate = float(es.sigma), float(es.lrate)
    pre_state, pre_step = agents.state.cpu().numpy(), agents.step.cpu().numpy()
    lev = agents.levels.cpu().numpy()
    spec = olv.env_spec(mode)
    p_lv, lt = olv.reset_env_params(jr.split(jr.split(jr.PRNGKey(1), 2)[1], N), mode)
    assert np.array_equal(olv.pack_levels(p_lv, lt, spec), lev)
    step.trace = []
    rng = jr.PRNGKey(13)
    m = step(prng.from_uint32_numpy(rng, "cuda"), agents)
    torch.cuda.synchronize()
    cur = step.cur
    # ---- population properties
    f = step.fitness.cpu().numpy()
    assert np.all(np.isfinite(f))
    rank, fg = oes.pair_rank(f)
    winners = np.where(fg, np.arange(N) * 2, np.arange(N) * 2 + 1)
    wi = torch.from_numpy(winners).cuda()
    assert torch.equal(agents.theta, step.theta[cur][wi]) and torch.equal(agents.phi, step.phi[cur][wi])
    assert float(m["fitness"]["mean"]) == pytest.approx(float(f.mean()), rel=1e-6, abs=1e-9)
    # ---- the tell gradient (float64 on the device: 1024 x 205,482 population)
    x = step.x
    g_ref = ((x.double() - pre_mean.double()) / pre_sigma).T @ (-torch.from_numpy(rank).cuda().double())
    g_ref = g_ref / (C * pre_sigma)
    g_dev = es.grad.double() / (es.popsize * pre_sigma)
    rel = float(torch.linalg.norm(g_dev - g_ref) / torch.linalg.norm(g_ref))
    assert rel <= 1e-6, rel
    st = {"mean": pre_mean.cpu().numpy().astype(np.float64), "m": pre_m.astype(np.float64),
          "v": pre_v.astype(np.float64), "n": pre_n, "lrate": pre_lrate, "sigma": pre_sigma,
          "lrate_decay": args.es_lrate_decay, "lrate_limit": args.es_lrate_limit, "sigma_decay": args.es_sigma_decay,
          "sigma_limit": args.es_sigma_limit}
    st = oes.opt_step(g_dev.cpu().numpy(), st, args.lpg_opt.lower())
    np.testing.assert_allclose(es.mean.cpu().numpy(), st["mean"], rtol=1e-6, atol=2e-8)
    # ---- sampled candidates: ask, rollouts, updates and fitness against the oracle
    xs = x[list(SAMPLED)].cpu().numpy()
    r1, sub = jr.split(rng, 2)
    # (the oracle's ask for the sampled rows: the antithetic pairs of rows c // 2)
    ask_ref = oes.ask(sub, pre_mean.cpu().numpy(), np.float32(pre_sigma), C)
    np.testing.assert_array_equal(xs, ask_ref[list(SAMPLED)])
    _, sub2 = jr.split(r1, 2)
    ck2 = jr.split(jr.split(sub2, C), 2)
    fit_keys, tk = ck2[:, 0], ck2[:, 1]
    sel = np.array(SAMPLED)
    agent_of = sel // 2
    p_sel = {kk: v[agent_of] for kk, v in p_lv.items()}
    rows = np.concatenate([np.arange(a * W, (a + 1) * W) for a in agent_of])
    ost = _state_np(torch.from_numpy(pre_state[:, rows]), spec)
    hyp = ometa.Hypers(lifetime_conditioning=True)
    th_k = [r["theta"][wi.new_tensor(sel)].cpu().numpy() for r in step.trace] + [step.theta[cur][wi.new_tensor(sel)].cpu().numpy()]
    ph_k = [r["phi"][wi.new_tensor(sel)].cpu().numpy() for r in step.trace] + [step.phi[cur][wi.new_tensor(sel)].cpu().numpy()]
    s = pre_step[agent_of].astype(np.int64)
    for k in range(K):
        s2 = jr.split(tk, 2)
        tk, rk = s2[:, 0], s2[:, 1]
        otr, ost, _ = oro.batch_rollout(spec, rk[sel], th_k[k], p_sel, ost, T)
        tr = step.trace[k]["traj"]
        for name, got in (("idx", tr.obs_idx), ("time", tr.obs_time), ("action", tr.action), ("reward", tr.reward),
                          ("done", tr.done)):
            g = got[wi.new_tensor(sel)].cpu().numpy()
            np.testing.assert_array_equal(g, otr[name].transpose(0, 2, 1).astype(g.dtype), err_msg=f"rollout {k} {name}")
        for i, c in enumerate(SAMPLED):
            tr_c = {"idx": otr["idx"][i], "time": otr["time"][i], "action": otr["action"][i].astype(np.int64),
                    "reward": otr["reward"][i], "done": otr["done"][i].astype(bool)}
            th = torch.tensor(th_k[k][i], dtype=torch.float64, requires_grad=True)
            ph = torch.tensor(ph_k[k][i], dtype=torch.float64, requires_grad=True)
            eta_c = torch.tensor(xs[i], dtype=torch.float64)
            th1, ph1, s_new, _, _ = ometa.lpg_agent_step(th, ph, int(s[i]), int(lev[agent_of[i], L_LIFETIME]), eta_c,
                                                        tr_c, hyp)
            s[i] = s_new
            for got0, got1, ref1, nm in ((th_k[k][i], th_k[k + 1][i], th1, "theta"),
                                         (ph_k[k][i], ph_k[k + 1][i], ph1, "phi")):
                d_ref = ref1.detach().numpy() - got0
                d_dev = got1.astype(np.float64) - got0
                assert np.linalg.norm(d_dev - d_ref) <= 2e-5 * np.linalg.norm(d_ref) + 1e-7, (nm, c, k)
    fit_ref = oag.eval_agent(spec, fit_keys[sel], p_sel, th_k[K], W, smp.max_rollout_len)
    np.testing.assert_allclose(f[sel], fit_ref, atol=1e-5)
    # the kept agents' steps and env states: the winners' (candidate c's state after its K rollouts)
    st_dev = agents.state.cpu().numpy().reshape(12, N, W)
    for i, c in enumerate(SAMPLED):
        a = c // 2
        if winners[a] != c:
            continue
        assert int(agents.step[a]) == int(s[i]), c
        got = _state_np(torch.from_numpy(st_dev[:, a]), spec)
        for kname in ("time", "pos", "obj_existss", "early_term", "obj_poss"):
            np.testing.assert_array_equal(got[kname], ost[kname][i * W:(i + 1) * W], err_msg=f"{c} {kname}")
