"""GPU parity of the LPG meta-gradient step vs the float64 torch-autograd oracle (oracle/meta.py).

The HIP step runs K inner LPG updates (fused rollout, MFMA GRU, clipped SGD), the
eval rollout and the explicit-adjoint meta-gradient.  The oracle replays the
same trajectories — every one of the K train rollouts and the eval rollout is
re-generated bit-exactly by the numpy rollout from the GPU's theta_k, the
oracle's own key chain (meta/train.py:41,47; lpg_agent.py:107) and the env state
carried from the previous rollout — and differentiates with autograd
(create_graph through the clipped SGD steps, stop_gradient on the LPG inputs as
in agents/lpg_agent.py:47-56).

Tolerances (float32 GPU vs float64 oracle), set a few times above the achieved
error so that a lost split-precision piece (~2^-11 relative) fails them: agent
parameters after K updates rtol/atol 2e-5; metrics rtol 2e-5; meta-gradient
relative L2 error < 1e-5; GRU forward outputs and saves 5e-6 abs; GRU backward
gradients 1e-5 relative L2.
"""
import os

import numpy as np
import pytest
import torch

from oracle import jaxrand as jr
from oracle import lpg as olpg
from oracle import meta as ometa
from oracle import rollout as oro
from oracle import levels as olv

pytestmark = pytest.mark.gpu


def _setup(mode, N, W, T, K, lifetime_conditioning=False, seed=0):
    from toued import prng
    from toued.agents import AgentBatch, create_agents, create_value_critics
    from toued.env import LevelGenerator
    from toued.lpg import init_lpg_params
    from toued.meta import AdamState, LpgHyperparams, MetaGradStep
    from toued.rollout import RolloutWrapper
    dk = lambda a: prng.from_uint32_numpy(a, "cuda")
    keys = jr.split(jr.PRNGKey(seed), N)
    gen = LevelGenerator(mode)
    levels = gen(dk(keys))
    ro = RolloutWrapper(mode, T, env_workers=W)
    D = ro.obs_dim
    theta, phi = create_agents(dk(jr.split(jr.PRNGKey(seed + 1), N)), D, 8)
    # sharpen the random init a little so policies are not uniform
    theta.mul_(30.0)
    phi.mul_(30.0)
    vcrit = create_value_critics(dk(jr.split(jr.PRNGKey(seed + 2), N)), D) * 30.0
    (_, _), state = ro.batch_reset(dk(jr.split(jr.PRNGKey(seed + 3), N)), levels)
    agents = AgentBatch(levels, theta, phi, torch.zeros(N, dtype=torch.int32, device="cuda"), state, vcrit,
                        torch.zeros(N, dtype=torch.int32, device="cuda"))
    hyp = LpgHyperparams(num_agent_updates=K)
    step = MetaGradStep(ro, N, hyp, lifetime_conditioning)
    F = 7 if lifetime_conditioning else 5
    eta = init_lpg_params(seed + 4, F)
    adam = AdamState(eta.numel(), "cuda")
    return agents, step, eta, adam, hyp, D


@pytest.mark.parametrize("mode,lc", [("dense", False), ("tabular", True), ("mazes", False), ("all_vrandlife", True)])
def test_meta_step_matches_oracle(mode, lc):
    N, W, T, K = 3, 64, 20, 3
    agents, step, eta, adam, hyp, D = _setup(mode, N, W, T, K, lc)
    theta0 = agents.theta.cpu().numpy()
    phi0 = agents.phi.cpu().numpy()
    vcrit = agents.vcrit.cpu().numpy()
    state0 = agents.state.cpu().numpy()
    eta0 = eta.clone()
    lv = agents.levels.cpu().numpy()
    rng = torch.tensor([0, 77], dtype=torch.int32, device="cuda")
    metrics = step(rng, eta, adam, agents)
    torch.cuda.synchronize()
    g_gpu = step.grad.cpu().double().numpy() / N   # f64: a float32 norm alone is off by ~1e-7 (the cosine bound is 1e-9)
    tr = step.traj
    idx = tr.obs_idx.cpu().numpy()
    tm = tr.obs_time.cpu().numpy()
    act = tr.action.cpu().numpy()
    rew = tr.reward.cpu().numpy()
    dn = tr.done.cpu().numpy()
    th_h = step.theta_h.cpu().numpy()
    th_h[0] = theta0          # slot 0 is the agents' own table storage: after the step it holds theta_K
    # ---- trajectories: every rollout k = 0..K bit-exact vs the numpy rollout driven by the GPU's theta_k
    spec = olv.env_spec(mode)
    keys = jr.split(jr.PRNGKey(0), N)
    p, lt = olv.reset_env_params(keys, mode)
    from test_gpu_env import _state_np
    ost = _state_np(torch.from_numpy(state0), spec)
    # meta/train.py:41 (r0, t) = split(rng_a); lpg_agent.py:107 (t, roll_k) = split(t) per update k;
    # meta/train.py:47 (r0, roll_eval) = split(r0)
    ka = jr.split(np.array([0, 77], np.uint32), N)
    r0t = jr.split(ka, 2)
    r0, tk = r0t[:, 0], r0t[:, 1]
    for k in range(K + 1):
        if k < K:
            s2 = jr.split(tk, 2)
            tk, rk = s2[:, 0], s2[:, 1]
        else:
            rk = jr.split(r0, 2)[:, 1]
        otr, ost, _ = oro.batch_rollout(spec, rk, th_h[k], p, ost, T)
        for name, got in (("idx", idx), ("time", tm), ("action", act), ("reward", rew), ("done", dn)):
            np.testing.assert_array_equal(got[k], otr[name].transpose(0, 2, 1).astype(got.dtype),
                                          err_msg=f"rollout {k} {name}")
    # ---- oracle meta-gradient on the same trajectories
    def tr_of(k, a):
        return {"idx": idx[k, a].T.copy(), "time": tm[k, a].T.copy(), "action": act[k, a].T.astype(np.int64),
                "reward": rew[k, a].T.copy(), "done": dn[k, a].T.astype(bool)}
    agents_o = []
    for a in range(N):
        agents_o.append(dict(theta=theta0[a], phi=phi0[a], vcrit=vcrit[a][:, None], step=0,
                             lifetime=int(lv[a, 5]), trajs=[tr_of(k, a) for k in range(K)], eval=tr_of(K, a)))
    ohyp = ometa.Hypers(lifetime_conditioning=lc)
    g_ref, aux, _ = ometa.meta_gradient(eta0.cpu().numpy().astype(np.float64), agents_o, ohyp, K)
    # parameters after K updates
    for a in range(N):
        np.testing.assert_allclose(agents.theta[a].cpu().numpy(), aux[a]["theta"], rtol=2e-5, atol=2e-5)
        np.testing.assert_allclose(agents.phi[a].cpu().numpy(), aux[a]["phi"], rtol=2e-5, atol=2e-5)
    lpg_ref = np.array([x["lpg_loss"] for x in aux])
    np.testing.assert_allclose(metrics["lpg_loss"].cpu().numpy(), lpg_ref, rtol=2e-5, atol=1e-7)
    for key in ("policy_entropy", "critic_entropy", "policy_l2", "critic_l2", "critic_loss"):
        ref = np.array([x["lpg_agent"][key] for x in aux])
        np.testing.assert_allclose(metrics["lpg_agent"][key].cpu().numpy(), ref, rtol=2e-5, atol=1e-7, err_msg=key)
    err = np.linalg.norm(g_gpu - g_ref) / np.linalg.norm(g_ref)
    cos = float(g_gpu @ g_ref / (np.linalg.norm(g_gpu) * np.linalg.norm(g_ref)))
    print(f"meta-gradient rel L2 {err:.2e}, cosine {cos:.9f}")
    assert err < 1e-5 and cos > 1 - 1e-9, (err, cos)


def test_gru_forward_matches_oracle():
    """LPG forward (MFMA GRU + heads) on random inputs vs the float64 oracle."""
    from toued.lpg import LPGGRU, LPGLayout, init_lpg_params
    N, W, T, K = 2, 64, 20, 1
    R = N * W
    lay = LPGLayout(5)
    eta = init_lpg_params(3, 5)
    torch.manual_seed(0)   # the perturbation must not depend on what earlier tests drew
    eta += torch.randn_like(eta) * 0.05
    gru = LPGGRU(lay, R, T, K, W, "cuda")
    gru.pack(eta)
    rs = np.random.RandomState(0)
    X = gru.X
    X.copy_(torch.from_numpy(rs.randn(5, K, T, R).astype(np.float32)))
    done = (rs.rand(K, N, T, W) < 0.1).astype(np.uint8)
    X[1, 0] = torch.from_numpy(done[0].transpose(1, 0, 2).reshape(T, R).astype(np.float32)).cuda()
    pi_hat = torch.zeros(K, T, R, device="cuda")
    y_hat = torch.zeros(K, T, 8, R, device="cuda")
    gru.forward(0, X, torch.from_numpy(done[0]).cuda(), eta, pi_hat, y_hat)
    torch.cuda.synchronize()
    # oracle: run the GRU core with x given directly
    P = olpg.unflatten(torch.tensor(eta.cpu().numpy(), dtype=torch.float64), 5)
    x = torch.tensor(X[:, 0].cpu().numpy(), dtype=torch.float64).permute(2, 1, 0)   # [R, T, F]
    d = torch.tensor(done[0].transpose(0, 2, 1).reshape(R, T).astype(bool))
    h = torch.zeros(R, 256, dtype=torch.float64)
    outs = [None] * T
    saved = {"hin": [None] * T, "r": [None] * T, "z": [None] * T, "n": [None] * T}
    for t in reversed(range(T)):
        h = torch.where(d[:, t, None], torch.zeros_like(h), h)
        xt = x[:, t]
        rg = torch.sigmoid(xt @ P["ir_w"] + P["ir_b"] + h @ P["hr_w"])
        zg = torch.sigmoid(xt @ P["iz_w"] + P["iz_b"] + h @ P["hz_w"])
        hn = h @ P["hn_w"] + P["hn_b"]
        ng = torch.tanh(xt @ P["in_w"] + P["in_b"] + rg * hn)
        saved["hin"][t], saved["r"][t], saved["z"][t], saved["n"][t] = h, rg, zg, ng
        saved.setdefault("hn", [None] * T)[t] = hn
        h = (1 - zg) * ng + zg * h
        outs[t] = h
    hs = torch.relu(torch.stack(outs, 1))
    pi_ref = (hs @ P["pi_w"] + P["pi_b"])[..., 0]
    y_ref = torch.softmax(hs @ P["y_w"] + P["y_b"], -1)
    np.testing.assert_allclose(pi_hat[0].cpu().numpy().T, pi_ref.numpy(), atol=5e-6, rtol=0)
    np.testing.assert_allclose(y_hat[0].cpu().numpy().transpose(2, 0, 1), y_ref.numpy(), atol=5e-6, rtol=0)
    # the saves the backward reads: [unit][column t*R + r]
    def tr(a):
        return a.reshape(256, T, R).transpose(1, 2, 0)
    # (the split-precision pair k_gru_fwd6 / k_gru_bwd6n saves no n: the backward recomputes it, gru.hip gate_n)
    from toued import _lib
    saves = [("hin", tr(gru.hin_rows().cpu().numpy())), ("r", tr(gru.s_rows(0).cpu().numpy())),
             ("z", tr(gru.s_rows(1).cpu().numpy())), ("hn", tr(gru.s_rows(3).cpu().numpy()))]
    if not _lib.lib().toued_gru_bwd_col_exp(R):
        saves.append(("n", tr(gru.S[2].cpu().numpy())))
    for name, arr in saves:
        ref = np.stack([saved[name][t].numpy() for t in range(T)])
        np.testing.assert_allclose(arr, ref, atol=5e-6 * (1 + np.abs(ref).max()), rtol=0, err_msg=name)


@pytest.mark.parametrize("N,W,gscale,wscale", [(2, 64, 1.0, 1.0), (3, 32, 1.0, 1.0), (2, 64, 1e12, 1.0),
                                               (2, 64, 1e-12, 1.0), (2, 64, 1.0, 4.0), (2, 64, 1.0, 1e-3)])
def test_gru_backward_matches_autograd(N, W, gscale, wscale):
    """LPG GRU VJP (toued_gru_bwd + the weight-gradient GEMMs over the saved m-major operands) vs float64
    torch autograd of the same GRU + heads: every GRU / head parameter gradient and the input cotangents
    dX3, dX4 within 1e-5 relative L2 (achieved 1e-7..2e-6; one dropped fp16 piece costs ~5e-4).

    relu kinks: the heads read relu(h_out) (models/lpg.py:81), whose derivative jumps at 0.  Where |h_out| is
    within float32 rounding of 0 the device and float64 may take different branches; at wscale 4 or 1e-3 ONE such
    flip in 393k elements moves the recurrent-fed gradients by 1e-3 relative (tools/gru_seed_sweep.py: 6 of 450
    seeded inputs, each with exactly one flip at |h| <= 1.4e-6, reruns bit-identical, 2e-6 with the device's branch
    -- this was the "intermittent" round-2 failure: the eta perturbation was unseeded then).  So the float64
    reference takes the device's relu decisions, every differing decision must lie within 5e-6 of the kink (the
    forward's own tolerance), and the flips are counted.  R = 128 runs the lockstep split-precision kernel, R = 96 (not a
    multiple of 64) the f32 kernel.  gscale multiplies the head cotangents (the backward's per-row fp16
    scales must follow them over 24 decades), wscale the recurrent weights W_hr, W_hz, W_hn (the per-unit
    weight scales of the forward and backward packs).  (At wscale 16 the gates saturate and the f32-MFMA kernel
    itself misses 1e-4 against float64: 1 - n^2 loses its digits in f32.)"""
    from toued.lpg import LPGLayout, init_lpg_params
    T, K, F = 6, 2, 5
    R = N * W
    lay = LPGLayout(F)
    eta = init_lpg_params(5, F)
    torch.manual_seed(0)   # the perturbation must not depend on what earlier tests drew
    eta += torch.randn_like(eta) * 0.05
    for name in ("hr_w", "hz_w", "hn_w"):
        lay.view(eta, name).mul_(wscale)
    rs = np.random.RandomState(1)
    xs = rs.randn(F, K, T, R).astype(np.float32)
    done = (rs.rand(K, N, T, W) < 0.15).astype(np.uint8)
    d_pi = (rs.randn(K, T, R) * gscale).astype(np.float32)
    d_y = (rs.randn(K, T, 8, R) * gscale).astype(np.float32)
    errs, flips = _gru_bwd_case(N, W, T, K, F, eta, xs, done, d_pi, d_y)
    tol = 1e-5 if R % 64 == 0 else 1e-4     # the f32-MFMA fallback (R % 64 != 0) keeps the f32 bound
    bad = {k: v for k, v in errs.items() if not v < tol}
    assert not bad, errs


@pytest.mark.parametrize("seed,wscale", [(129, 4.0), (104, 1e-3)])
def test_gru_backward_relu_kink_inputs(seed, wscale):
    """The inputs of tools/gru_seed_sweep.py seeds that flip one relu decision (|h_out| 5.4e-7 at wscale 4,
    5.1e-8 at wscale 1e-3; recurrent-fed gradients 2.9e-3 / 5.1e-3 off the float64 branch): with the device's
    branch the backward is within 1e-5, and the flip sits inside the kink band."""
    from toued.lpg import LPGLayout, init_lpg_params
    N, W, T, K, F = 2, 64, 6, 2, 5
    R = N * W
    lay = LPGLayout(F)
    eta0 = init_lpg_params(5, F)
    g = torch.Generator(device="cpu").manual_seed(seed)
    eta = eta0.clone() + (torch.randn(eta0.shape, generator=g) * 0.05).cuda()
    for name in ("hr_w", "hz_w", "hn_w"):
        lay.view(eta, name).mul_(wscale)
    rs = np.random.RandomState(100000 + seed)
    xs = rs.randn(F, K, T, R).astype(np.float32)
    done = (rs.rand(K, N, T, W) < 0.15).astype(np.uint8)
    d_pi = rs.randn(K, T, R).astype(np.float32)
    d_y = rs.randn(K, T, 8, R).astype(np.float32)
    errs, flips = _gru_bwd_case(N, W, T, K, F, eta, xs, done, d_pi, d_y)
    assert len(flips) >= 1
    assert max(errs.values()) < 1e-5, errs


def _gru_bwd_case(N, W, T, K, F, eta, xs, done, d_pi, d_y):
    """forward + backward + weight gradients on the device; float64 autograd with the device's relu branches;
    relative L2 errors per parameter and of dX3/dX4, and |h_out| of every relu decision taken from the device."""
    from toued.lpg import LPGGRU, LPGLayout
    R = N * W
    lay = LPGLayout(F)
    gru = LPGGRU(lay, R, T, K, W, "cuda")
    gru.keep_inputs = True      # relu_out() below
    gru.pack(eta)
    gru.X.copy_(torch.from_numpy(xs))
    X = gru.X
    done_t = torch.from_numpy(done).cuda()
    pi_hat = torch.zeros(K, T, R, device="cuda")
    y_hat = torch.zeros(K, T, 8, R, device="cuda")
    for k in range(K):
        gru.forward(k, X, done_t[k], eta, pi_hat, y_hat)
    grad = torch.zeros(lay.size, device="cuda")
    gru.backward(done_t, eta, y_hat, torch.from_numpy(d_pi).cuda(), torch.from_numpy(d_y).cuda(), X, grad)
    torch.cuda.synchronize()
    # float64 autograd oracle, relu branches from the device (RH = relu(h_out) rows [256][M], column (k, t, r))
    relu_dev = (gru.relu_out() > 0).cpu().numpy().reshape(256, K, T, R)
    flips = []
    flat = torch.tensor(eta.cpu().numpy(), dtype=torch.float64, requires_grad=True)
    P = olpg.unflatten(flat, F)
    x = torch.tensor(xs, dtype=torch.float64, requires_grad=True)       # [F, K, T, R]
    loss = 0.0
    for k in range(K):
        xk = x[:, k].permute(2, 1, 0)                                     # [R, T, F]
        d = torch.tensor(done[k].transpose(0, 2, 1).reshape(R, T).astype(bool))
        h = torch.zeros(R, 256, dtype=torch.float64)
        outs = [None] * T
        for t in reversed(range(T)):
            h = torch.where(d[:, t, None], torch.zeros_like(h), h)
            xt = xk[:, t]
            rg = torch.sigmoid(xt @ P["ir_w"] + P["ir_b"] + h @ P["hr_w"])
            zg = torch.sigmoid(xt @ P["iz_w"] + P["iz_b"] + h @ P["hz_w"])
            ng = torch.tanh(xt @ P["in_w"] + P["in_b"] + rg * (h @ P["hn_w"] + P["hn_b"]))
            h = (1 - zg) * ng + zg * h
            outs[t] = h
        hst = torch.stack(outs, 1)                                         # [R, T, 256]
        mk = torch.from_numpy(relu_dev[:, k].transpose(2, 1, 0).copy())    # [R, T, 256]
        hv = hst.detach().numpy()
        flips.extend(np.abs(hv[mk.numpy() != (hv > 0)]).tolist())
        hs = torch.where(mk, hst, torch.zeros_like(hst))
        pi_ref = (hs @ P["pi_w"] + P["pi_b"])[..., 0]                      # [R, T]
        y_ref = torch.softmax(hs @ P["y_w"] + P["y_b"], -1)                # [R, T, 8]
        dpi = torch.tensor(d_pi[k].T, dtype=torch.float64)
        dy = torch.tensor(d_y[k].transpose(2, 0, 1), dtype=torch.float64)
        loss = loss + (pi_ref * dpi).sum() + (y_ref * dy).sum()
    loss.backward()
    g_ref = flat.grad.numpy()
    g = grad.cpu().numpy().astype(np.float64)
    errs = {}
    for name in ("hr_w", "hz_w", "hn_w", "ir_w", "iz_w", "in_w", "ir_b", "iz_b", "in_b", "hn_b", "pi_w", "pi_b",
                 "y_w", "y_b"):
        o = lay.offsets[name]
        sl = slice(o, o + int(np.prod(lay.shapes[name])))
        errs[name] = np.linalg.norm(g[sl] - g_ref[sl]) / max(np.linalg.norm(g_ref[sl]), 1e-300)
    gx = x.grad.numpy()
    for f, dX in ((3, gru.dX3), (4, gru.dX4)):
        got = dX.cpu().numpy()
        errs[f"dX{f}"] = np.linalg.norm(got - gx[f]) / np.linalg.norm(gx[f])
    print("gru backward relative L2 errors:", {k: f"{v:.2e}" for k, v in errs.items()},
          f"relu decisions taken from the device: {len(flips)} (max |h_out| {max(flips, default=0.0):.1e})")
    assert all(f < 5e-6 for f in flips), flips
    return errs, flips


def test_gru_backward_repeat_bit_identical():
    """Two backward passes over the same saved activations give bit-identical outputs: the kernels have no
    atomics and fixed reduction orders, so any difference is a race (this caught a lane-half LDS hazard in the
    input-cotangent partials of k_gru_bwd6)."""
    from toued.lpg import LPGGRU, LPGLayout, init_lpg_params
    N, W, T, K, F = 2, 64, 6, 2, 5
    R = N * W
    lay = LPGLayout(F)
    eta = init_lpg_params(7, F)
    gru = LPGGRU(lay, R, T, K, W, "cuda")
    gru.pack(eta)
    rs = np.random.RandomState(2)
    gru.X.copy_(torch.from_numpy(rs.randn(F, K, T, R).astype(np.float32)))
    done_t = torch.from_numpy((rs.rand(K, N, T, W) < 0.15).astype(np.uint8)).cuda()
    pi_hat = torch.zeros(K, T, R, device="cuda")
    y_hat = torch.zeros(K, T, 8, R, device="cuda")
    for k in range(K):
        gru.forward(k, gru.X, done_t[k], eta, pi_hat, y_hat)
    d_pi = torch.from_numpy(rs.randn(K, T, R).astype(np.float32)).cuda()
    d_y = torch.from_numpy(rs.randn(K, T, 8, R).astype(np.float32)).cuda()
    outs = []
    for _ in range(3):
        gru.dX3.fill_(float("nan"))
        gru.dX4.fill_(float("nan"))
        grad = torch.zeros(lay.size, device="cuda")
        gru.backward(done_t, eta, y_hat, d_pi, d_y, gru.X, grad)
        torch.cuda.synchronize()
        outs.append([gru.dX3.clone(), gru.dX4.clone(), gru.DG[:3].clone(), gru.GI.clone(), grad])
    for rep in outs[1:]:
        for a, b in zip(outs[0], rep):
            assert torch.isfinite(a).all()
            assert torch.equal(a, b)


@pytest.mark.parametrize("N,W,wscale", [(2, 64, 4.0), (40, 64, 1.0)])
def test_gru_independent_of_scratch_contents(N, W, wscale):
    """Forward + backward + weight gradients give bit-identical results whatever the scratch buffers held
    before (zeros, NaN, random bits): no kernel reads a save, cotangent, partial or workspace element it has not
    written in the same pass.  The open intermittent failure of test_gru_backward_matches_autograd[2-64-1.0-4.0]
     depended on what earlier tests left in the caching allocator if it was such a read; this makes
    the dependence deterministic instead of luck.  N=40 gives 40 row groups so workgroups run concurrently."""
    from toued.lpg import H, LPGGRU, LPGLayout, init_lpg_params
    T, K, F = 6, 2, 5
    R = N * W
    lay = LPGLayout(F)
    eta = init_lpg_params(5, F)
    torch.manual_seed(0)   # the perturbation must not depend on what earlier tests drew
    eta += torch.randn_like(eta) * 0.05
    for name in ("hr_w", "hz_w", "hn_w"):
        lay.view(eta, name).mul_(wscale)
    rs = np.random.RandomState(3)
    xs = torch.from_numpy(rs.randn(F, K, T, R).astype(np.float32)).cuda()
    done_t = torch.from_numpy((rs.rand(K, N, T, W) < 0.15).astype(np.uint8)).cuda()
    d_pi = torch.from_numpy(rs.randn(K, T, R).astype(np.float32)).cuda()
    d_y = torch.from_numpy(rs.randn(K, T, 8, R).astype(np.float32)).cuda()
    gen = torch.Generator(device="cuda").manual_seed(11)

    def fill(t, how):
        if how == "zero":
            t.zero_()
        elif how == "nan":
            t.view(torch.int8 if t.dtype == torch.int8 else torch.int32).fill_(-1)   # all-ones bits: NaN / -1
        else:
            b = t.view(torch.uint8)
            b.copy_(torch.randint(0, 256, b.shape, generator=gen, device="cuda", dtype=torch.uint8))

    outs = {}
    for how in ("zero", "nan", "random", "zero"):
        gru = LPGGRU(lay, R, T, K, W, "cuda")
        # (fwdA / bwdA: the packed weights, whose unused piece slots the pack kernels leave unwritten)
        bufs = [gru.S, gru.DG, gru.dX3, gru.dX4, gru._ggi, gru.CE, gru.wg_work, gru.A[:H], gru.fwdA, gru.bwdA]
        if not gru.fused:
            bufs += [gru.DH, gru.RH[:H]]
        for t in bufs:
            if t.numel():
                fill(t, how)
        gru.pack(eta)
        gru.X.copy_(xs)
        pi_hat = torch.zeros(K, T, R, device="cuda")
        y_hat = torch.zeros(K, T, 8, R, device="cuda")
        for k in range(K):
            gru.forward(k, gru.X, done_t[k], eta, pi_hat, y_hat)
        grad = torch.zeros(lay.size, device="cuda")
        gru.backward(done_t, eta, y_hat, d_pi, d_y, gru.X, grad)
        torch.cuda.synchronize()
        got = [pi_hat, y_hat, gru.dX3.clone(), gru.dX4.clone(), grad]
        assert all(torch.isfinite(g).all() for g in got), how
        if "zero" in outs:
            for i, (a, b) in enumerate(zip(outs["zero"], got)):
                assert torch.equal(a, b), (how, i, (a - b).abs().max().item())
        else:
            outs["zero"] = got
        del gru


@pytest.mark.parametrize("extra", [[], ["--score_function", "alg_regret", "--env_mode", "all_shortlife"]])
def test_train_main_writes_checkpoints(tmp_path, extra):
    """train.py driver end to end (2 meta-steps) with --checkpoint_dir: the restored TrainState holds the
    trainer's final LPG parameters and Adam state; buffer-based score functions also write buffer_<steps>."""
    from toued import train
    from toued.checkpoint import lpg_flat_from_tree, restore_checkpoint
    from toued.lpg import LPGLayout
    argv = ["--env_mode", "tabular", "--num_agents", "2", "--num_mini_batches", "1", "--train_steps", "2",
            "--checkpoint_dir", str(tmp_path)] + extra
    captured = {}
    orig = train.save_final_checkpoints

    def spy(ckpt_dir, tr, steps):
        captured["eta"], captured["m"] = tr.eta.cpu().numpy().copy(), tr.adam.m.cpu().numpy().copy()
        orig(ckpt_dir, tr, steps)
    train.save_final_checkpoints = spy
    try:
        train.main(argv)
    finally:
        train.save_final_checkpoints = orig
    r = restore_checkpoint(str(tmp_path))
    lay = LPGLayout(5)
    assert int(r["step"]) == 2 and int(r["opt_state"]["0"]["count"]) == 2
    assert np.array_equal(lpg_flat_from_tree(r["params"], lay), captured["eta"])
    assert np.array_equal(lpg_flat_from_tree(r["opt_state"]["0"]["mu"], lay), captured["m"])
    files = sorted(os.listdir(tmp_path))
    assert files == (["buffer_2", "checkpoint_2"] if extra else ["checkpoint_2"])
    if extra:
        b = restore_checkpoint(str(tmp_path), prefix="buffer_")
        assert b["level"]["env_params"]["walls"].shape == (4000, 100) and b["score"].dtype == np.float32
        assert b["level"]["env_params"]["obj_rewards"].shape == (4000, 5)


def _agents_for(mode, N, W, T, seed):
    from toued import prng
    from toued.agents import AgentBatch, create_agents, create_value_critics
    from toued.env import LevelGenerator
    from toued.rollout import RolloutWrapper
    dk = lambda a: prng.from_uint32_numpy(a, "cuda")
    levels = LevelGenerator(mode)(dk(jr.split(jr.PRNGKey(seed), N)))
    ro = RolloutWrapper(mode, T, env_workers=W)
    theta, phi = create_agents(dk(jr.split(jr.PRNGKey(seed + 1), N)), ro.obs_dim, 8)
    vcrit = create_value_critics(dk(jr.split(jr.PRNGKey(seed + 2), N)), ro.obs_dim)
    (_, _), state = ro.batch_reset(dk(jr.split(jr.PRNGKey(seed + 3), N)), levels)
    z = lambda: torch.zeros(N, dtype=torch.int32, device="cuda")
    return ro, AgentBatch(levels, theta, phi, z(), state, vcrit, z())


def _clone_agents(ag):
    from toued.agents import AgentBatch
    return AgentBatch(*(None if x is None else x.clone() for x in
                        (ag.levels, ag.theta, ag.phi, ag.step, ag.state, ag.vcrit, ag.vstep)))


@pytest.mark.parametrize("nmb", [2, 4])
def test_mini_batches_match_full_batch(nmb):
    """--num_mini_batches (util/jax.py:25-41 mini_batch_vmap, a numerical no-op): sequential agent chunks give
    bit-identical agents, env states and metrics, and the same summed meta-gradient up to the summation
    grouping (1e-6)."""
    from toued.lpg import init_lpg_params
    from toued.meta import AdamState, LpgHyperparams, MetaGradStep
    N, W, T, K = 8, 64, 20, 2
    ro, ag0 = _agents_for("dense", N, W, T, 70)
    eta0 = init_lpg_params(71, 5)
    rng = torch.tensor([0, 123], dtype=torch.int32, device="cuda")
    out = []
    for m in (1, nmb):
        ag = _clone_agents(ag0)
        eta = eta0.clone()
        step = MetaGradStep(ro, N, LpgHyperparams(num_agent_updates=K), False, num_mini_batches=m)
        met = step(rng, eta, AdamState(eta.numel(), "cuda"), ag)
        torch.cuda.synchronize()
        out.append((ag, step.grad.clone(), met, eta))
    (a1, g1, m1, e1), (a2, g2, m2, e2) = out
    for name in ("theta", "phi", "step", "state", "vstep"):
        assert torch.equal(getattr(a1, name), getattr(a2, name)), name
    for k in ("lpg_loss", "value_loss", "lpg_agent_return"):
        assert torch.equal(m1[k], m2[k]), k
    for k in m1["lpg_agent"]:
        assert torch.equal(m1["lpg_agent"][k], m2["lpg_agent"][k]), k
    assert float((g1 - g2).norm() / g1.norm()) < 1e-6
    assert float((e1 - e2).abs().max()) < 1e-7


@pytest.mark.parametrize("mode,N,lc", [("tabular", 512, False), ("all_vrandlife", 16, True)])
def test_fused_agent_step_matches_dense_path(monkeypatch, mode, N, lc):
    """The inner updates as toued_agent_step (theta_{k+1} copied on the side stream, touched rows rewritten,
    gradient rows kept; the reverse pass's entropy gradient and clip-VJP dot fused over those rows) against the
    dense toued_agent_grad + apply + entropy + clip_dot path, over two consecutive meta-steps (the second one's gradient tables hold the first one's rows
    where it does not write): every theta_k / phi_k, the agents, metrics and gstat bit-identical; the
    meta-gradient up to the clip-VJP dot's summation order (1e-6)."""
    from toued.lpg import init_lpg_params
    from toued.meta import AdamState, LpgHyperparams, MetaGradStep
    W, T, K = 64, 20, 5
    ro, ag0 = _agents_for(mode, N, W, T, 90)
    eta0 = init_lpg_params(91, 7 if lc else 5)
    out = []
    for fused in ("0", "1"):
        monkeypatch.setenv("TOUED_META_FUSED_STEP", fused)
        ag = _clone_agents(ag0)
        step = MetaGradStep(ro, N, LpgHyperparams(num_agent_updates=K), lc)
        assert step.fused_step == (fused == "1")
        hist = []
        for i in range(2):   # the same eta both times (Adam's step would carry the gradients' last-bit difference)
            eta = eta0.clone()
            met = step(torch.tensor([5, 60 + i], dtype=torch.int32, device="cuda"), eta,
                       AdamState(eta.numel(), "cuda"), ag)
            torch.cuda.synchronize()
            hist.append((step.theta_h.clone(), step.phi_h.clone(), step.gstat.clone(), step.grad.clone(), met))
        out.append((ag, hist))
    (a0, h0), (a1, h1) = out
    for name in ("theta", "phi", "step", "state", "vstep"):
        assert torch.equal(getattr(a0, name), getattr(a1, name)), name
    for (th0, ph0, gs0, g0, m0), (th1, ph1, gs1, g1, m1) in zip(h0, h1):
        assert torch.equal(th0, th1) and torch.equal(ph0, ph1)
        assert torch.equal(gs0, gs1)
        for k in m0["lpg_agent"]:
            assert torch.equal(m0["lpg_agent"][k], m1["lpg_agent"][k]), k
        for k in ("lpg_loss", "lpg_agent_return"):
            assert torch.equal(m0[k], m1[k]), k
        rel = float((g0 - g1).norm() / g0.norm())
        print(f"meta-gradient fused vs dense rel L2 {rel:.2e}")
        assert rel < 1e-6


@pytest.mark.parametrize("mode,N,lc", [("tabular", 512, False), ("all_vrandlife", 16, True)])
def test_one_launch_update_and_reverse_step_bit_identical(monkeypatch, mode, N, lc):
    """toued_agent_step_entropy (the inner update and its entropy metrics in one launch) and toued_entropy_clip_hvp
    (the reverse pass's entropy-clip and HVP of step k in one launch, one sort) against the separate launches
    (TOUED_STEP_ENTROPY=0, TOUED_REVERSE_PAIR=0), over two consecutive meta-steps: the meta-gradient, every
    theta_k / phi_k, the adjoint's cotangents d_pi_hat / d_y_hat, the agents and the metrics bit-identical."""
    from toued.lpg import init_lpg_params
    from toued.meta import AdamState, LpgHyperparams, MetaGradStep
    from toued.env import L_LIFETIME
    W, T, K = 64, 20, 5
    ro, ag0 = _agents_for(mode, N, W, T, 92)
    # every third agent two updates short of its lifetime: its later updates are not applied (HvpOp then keeps none
    # of its samples, the case where the one-launch reverse step's second op drops what the first op sorted)
    life = ag0.levels[:, L_LIFETIME]
    ag0.step[::3] = (life[::3] - 2).clamp(min=0).to(ag0.step.dtype)
    eta0 = init_lpg_params(93, 7 if lc else 5)
    out = []
    for one in ("0", "1"):
        monkeypatch.setenv("TOUED_STEP_ENTROPY", one)
        monkeypatch.setenv("TOUED_REVERSE_PAIR", one)
        ag = _clone_agents(ag0)
        step = MetaGradStep(ro, N, LpgHyperparams(num_agent_updates=K), lc)
        assert step.fused_step and step.step_entropy == (one == "1") and step.reverse_pair == (one == "1")
        hist = []
        for i in range(2):
            eta = eta0.clone()
            met = step(torch.tensor([7, 30 + i], dtype=torch.int32, device="cuda"), eta,
                       AdamState(eta.numel(), "cuda"), ag)
            torch.cuda.synchronize()
            hist.append((step.theta_h.clone(), step.phi_h.clone(), step.d_pi_hat.clone(), step.d_y_hat.clone(),
                         step.grad.clone(), met))
        out.append((ag, hist))
    (a0, h0), (a1, h1) = out
    for name in ("theta", "phi", "step", "state", "vstep"):
        assert torch.equal(getattr(a0, name), getattr(a1, name)), name
    for x0, x1 in zip(h0, h1):
        for j in range(5):
            assert torch.equal(x0[j], x1[j]), j
        m0, m1 = x0[5], x1[5]
        for k in m0["lpg_agent"]:
            assert torch.equal(m0["lpg_agent"][k], m1["lpg_agent"][k]), k
        for k in ("lpg_loss", "reg_lpg_loss", "lpg_agent_return"):
            assert torch.equal(m0[k], m1[k]), k


def test_1024_agents_two_mini_batches_on_one_gpu():
    """A reference-legal --num_agents 1024 --num_mini_batches 2 on one GPU (one 512-agent batch alone is the
    bench's size; 1024 at once exceeds the GRU kernels' 4 GiB operand range, so --num_mini_batches 1 runs the same
    two chunks): each chunk equals an unchunked
    512-agent step over the same agents and keys (rank_slice = the chunk of split(rng, 1024))."""
    from toued.lpg import init_lpg_params
    from toued.meta import AdamState, LpgHyperparams, MetaGradStep
    N, W, T, K = 1024, 64, 20, 5
    ro, ag0 = _agents_for("tabular", N, W, T, 80)
    eta0 = init_lpg_params(81, 5)
    rng = torch.tensor([3, 4], dtype=torch.int32, device="cuda")
    hyp = LpgHyperparams(num_agent_updates=K)
    ag = _clone_agents(ag0)
    eta = eta0.clone()
    big = MetaGradStep(ro, N, hyp, False, num_mini_batches=2)
    met = big(rng, eta, AdamState(eta.numel(), "cuda"), ag)
    torch.cuda.synchronize()
    g_big = big.grad.clone()
    assert torch.isfinite(g_big).all() and torch.isfinite(met["lpg_agent_return"]).all()
    del big
    # --num_mini_batches 1 with the same 1024 agents: past the kernels' range (meta.gru_max_agents = 635) the batch
    # runs as the same two chunks by itself, bit-identical
    one = MetaGradStep(ro, N, hyp, False, num_mini_batches=1)
    assert one.n_chunks == 2
    ag1 = _clone_agents(ag0)
    one(rng, eta0.clone(), AdamState(eta0.numel(), "cuda"), ag1)
    torch.cuda.synchronize()
    assert torch.equal(one.grad, g_big) and torch.equal(ag1.theta, ag.theta)
    del one, ag1
    half = MetaGradStep(ro, 512, hyp, False)
    g_sum = torch.zeros_like(g_big)
    for lo in (0, 512):
        sub = _clone_agents(ag0)
        from toued.agents import AgentBatch
        part = AgentBatch(sub.levels[lo:lo + 512].contiguous(), sub.theta[lo:lo + 512].contiguous(),
                          sub.phi[lo:lo + 512].contiguous(), sub.step[lo:lo + 512].contiguous(),
                          sub.state[:, lo * W:(lo + 512) * W].contiguous(), sub.vcrit[lo:lo + 512].contiguous(),
                          sub.vstep[lo:lo + 512].contiguous())
        half(rng, eta0.clone(), AdamState(eta0.numel(), "cuda"), part, (lo, lo + 512, N))
        torch.cuda.synchronize()
        g_sum += half.grad
        assert torch.equal(part.theta, ag.theta[lo:lo + 512])
        assert torch.equal(part.state, ag.state[:, lo * W:(lo + 512) * W])
    assert float((g_sum - g_big).norm() / g_big.norm()) < 1e-6


def test_fix_value_critic_matches_oracle():
    """--fix_value_critic (SURVEY B.3 fixed): the value critic takes K SGD updates on the train rollouts, the
    eval advantages / value loss use those parameters, then one update on the eval rollout — vs the float64
    oracle (oracle/meta.value_critic_step); the meta-gradient and agent tables as in the frozen case."""
    N, W, T, K = 3, 64, 20, 3
    agents, step, eta, adam, hyp, D = _setup("dense", N, W, T, K)
    step.hyp.fix_value_critic = True
    th0, ph0, vc0 = agents.theta.cpu().numpy(), agents.phi.cpu().numpy(), agents.vcrit.cpu().numpy()
    lv = agents.levels.cpu().numpy()
    eta0 = eta.cpu().numpy().astype(np.float64)
    metrics = step(torch.tensor([0, 41], dtype=torch.int32, device="cuda"), eta, adam, agents)
    torch.cuda.synchronize()
    tr = step.traj
    idx, tm, act = tr.obs_idx.cpu().numpy(), tr.obs_time.cpu().numpy(), tr.action.cpu().numpy()
    rew, dn = tr.reward.cpu().numpy(), tr.done.cpu().numpy()

    def tr_of(k, a):
        return {"idx": idx[k, a].T.copy(), "time": tm[k, a].T.copy(), "action": act[k, a].T.astype(np.int64),
                "reward": rew[k, a].T.copy(), "done": dn[k, a].T.astype(bool)}
    ags = [dict(theta=th0[a], phi=ph0[a], vcrit=vc0[a][:, None], step=0, lifetime=int(lv[a, 5]),
                trajs=[tr_of(k, a) for k in range(K)], eval=tr_of(K, a)) for a in range(N)]
    g_ref, aux, _ = ometa.meta_gradient(eta0, ags, ometa.Hypers(fix_value_critic=True), K)
    vc = agents.vcrit.cpu().numpy().astype(np.float64)
    for a in range(N):
        dv, dv_ref = vc[a] - vc0[a], aux[a]["vcrit"][:, 0] - vc0[a]
        assert np.linalg.norm(dv - dv_ref) <= 2e-5 * np.linalg.norm(dv_ref) + 1e-9, a
    assert agents.vstep.cpu().tolist() == [K + 1] * N
    np.testing.assert_allclose(metrics["value_loss"].cpu().numpy(), [x["value_loss"] for x in aux], rtol=2e-5)
    np.testing.assert_allclose(metrics["lpg_loss"].cpu().numpy(), [x["lpg_loss"] for x in aux], rtol=2e-5,
                               atol=1e-7)
    g = step.grad.cpu().numpy() / N
    assert np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref) < 1e-5


@pytest.mark.parametrize("F,per_agent", [(5, False), (7, True)])
def test_lpg_inputs_rows_bitexact(F, per_agent):
    """toued_lpg_inputs_rows (one thread per GRU row over its T steps, the next step's critic embedding reused) against
    the per-sample toued_lpg_inputs (models/lpg.py:48-77): the LPG input matrix bit-identical, with shared and
    per-agent (ES candidate) embedding parameters, episode ends (done) in the trajectories and a strided X."""
    from toued import _lib as L
    from toued.env import L_LIFETIME
    N, W, T, D = 6, 128, 20, 1937
    g = torch.Generator(device="cuda").manual_seed(F)
    theta = torch.randn(N, D, 5, generator=g, device="cuda") * 3
    phi = torch.randn(N, D, 8, generator=g, device="cuda") * 3
    tidx = torch.randint(0, D - 1, (N, T + 1, W), generator=g, device="cuda", dtype=torch.int32)
    ttime = torch.randint(0, 250, (N, T + 1, W), generator=g, device="cuda", dtype=torch.int32)
    tact = torch.randint(0, 5, (N, T, W), generator=g, device="cuda", dtype=torch.uint8)
    trew = torch.randn(N, T, W, generator=g, device="cuda")
    tdone = (torch.rand(N, T, W, generator=g, device="cuda") < 0.1).to(torch.uint8)
    ns = N if per_agent else 1
    stride = 161 if per_agent else 0
    eta = torch.randn(ns, 161, generator=g, device="cuda") * 0.5
    e1w, e1b, e2w, e2b = eta[:, 0:128], eta[:, 128:144], eta[:, 144:160], eta[:, 160:161]
    step = torch.randint(0, 100, (N,), generator=g, device="cuda", dtype=torch.int32)
    levels = torch.zeros(N, 80, dtype=torch.int32, device="cuda")
    levels[:, L_LIFETIME] = torch.randint(100, 3000, (N,), generator=g, device="cuda", dtype=torch.int32)
    R = N * W
    xs_col, xs_f = 2, 2 * T * R + 64
    outs = []
    for fn in ("toued_lpg_inputs", "toued_lpg_inputs_rows"):
        X = torch.full((F * xs_f,), float("nan"), device="cuda")
        L.call(fn, N, W, T, D, F, L.ptr(theta), L.ptr(phi), L.ptr(tidx), L.ptr(ttime), L.ptr(tact), L.ptr(trew),
               L.ptr(tdone), L.ptr(eta) + 0, L.ptr(eta) + 4 * 128, L.ptr(eta) + 4 * 144, L.ptr(eta) + 4 * 160,
               L.ptr(step), L.ptr(levels), L.ptr(X), xs_f, xs_col, stride, L.stream_ptr())
        torch.cuda.synchronize()
        outs.append(X)
    a, b = outs
    assert torch.isnan(a).sum() == torch.isnan(b).sum()      # the same elements written (strided X)
    m = ~torch.isnan(a)
    assert int(m.sum()) == F * T * R
    assert torch.equal(a[m], b[m])


@pytest.mark.parametrize("N,wscale,F", [(2, 4.0, 5), (12, 1.0, 5), (2, 1.0, 1), (2, 1.0, 6)])
def test_gru_backward_fused_small_matches_unfused(N, wscale, F):
    """k_gru_bwd6n<true> (the two small weight-gradient products accumulated in the kernel on 16x16x4 f32 MFMAs,
    reduced from per-workgroup partials) against the unfused pair k_gru_bwd6n<false> + toued_gru_bwd_small: the
    contraction cotangents, column exponents and input cotangents bit-identical (the same gate maths), the small
    products GI within 2e-6 relative (exact f32 products, another summation order), the flat gradient within 1e-6
    relative L2.  F = 1 (the ones row at A-table row 1) and F = 6 (head cotangent rows up to row 15, the table's last)
    are the edges of the A table's packing."""
    from toued.lpg import LPGGRU, LPGLayout, init_lpg_params
    W, T, K = 64, 6, 2
    R = N * W
    lay = LPGLayout(F, kernel_test=True)
    eta = init_lpg_params(7, F)
    gen = torch.Generator(device="cuda").manual_seed(5)
    eta += torch.randn(eta.shape, device="cuda", generator=gen) * 0.05
    for name in ("hr_w", "hz_w", "hn_w"):
        lay.view(eta, name).mul_(wscale)
    rs = np.random.RandomState(9)
    xs = torch.from_numpy(rs.randn(F, K, T, R).astype(np.float32)).cuda()
    done_t = torch.from_numpy((rs.rand(K, N, T, W) < 0.15).astype(np.uint8)).cuda()
    d_pi = torch.from_numpy(rs.randn(K, T, R).astype(np.float32)).cuda()
    d_y = torch.from_numpy(rs.randn(K, T, 8, R).astype(np.float32)).cuda()
    outs = []
    for fused in (False, True):
        gru = LPGGRU(lay, R, T, K, W, "cuda", fused=fused)
        assert gru.fused == fused
        gru.pack(eta)
        gru.X.copy_(xs)
        pi_hat = torch.zeros(K, T, R, device="cuda")
        y_hat = torch.zeros(K, T, 8, R, device="cuda")
        for k in range(K):
            gru.forward(k, gru.X, done_t[k], eta, pi_hat, y_hat)
        grad = torch.zeros(lay.size, device="cuda")
        gru.backward(done_t, eta, y_hat, d_pi, d_y, gru.X, grad)
        torch.cuda.synchronize()
        outs.append((gru.dg_rows()[:3].clone(), gru.CE.clone(), gru.dX3.clone(), gru.dX4.clone(), gru.GI.clone(),
                     grad))
    (dg0, ce0, x30, x40, gi0, g0), (dg1, ce1, x31, x41, gi1, g1) = outs
    assert torch.equal(dg0, dg1) and torch.equal(ce0, ce1)
    assert torch.equal(x30, x31) and torch.equal(x40, x41)
    gi0, gi1 = gi0.double(), gi1.double()
    # per block ([8][256] then [9][257]), elementwise against the block's scale
    for a, b in ((gi0[:8 * 256], gi1[:8 * 256]), (gi0[8 * 256:], gi1[8 * 256:])):
        assert float((a - b).abs().max()) <= 2e-6 * float(a.abs().max()), float((a - b).abs().max())
    g0, g1 = g0.double(), g1.double()
    assert float((g0 - g1).norm() / g0.norm()) < 1e-6
