"""The C2 hot path at its production size against float64 (meta/train.py:122-129, models/lpg.py:11-36 and its VJP).

One Trainer at BASELINE configs[1] -- env_mode=tabular, num_agents=512, num_mini_batches=1, K=5 inner updates,
W=64 workers, T=20: M = K*T*N*W = 3,276,800 GRU columns -- runs meta-steps in production order (eval_agent's env
chain beside k_wgrad_h3, TOUED_EVAL_KEYS_EARLY default).  After the last step the operands the kernels left in HBM
are checked:

* the main weight-gradient product G = [h_in; x; 1] . [dr; dz; dhn]^T (k_wgrad_h3 on block-floating-point fp16 pairs,
  262 x 768 over M columns) against a float64 GEMM of the same f32 operands on the GPU: elementwise at the
  test_gpu_wgrad.py bound |C - C64| <= 2e-6 sqrt(M) (|A| . |B|^T), and relative L2 over the whole matrix < 1e-5 (a
  K chunk claimed twice or skipped moves it by ~1/sqrt(chunks), far above that);
* every tile of that launch claimed exactly once from k_wgrad_h3's per-XCD queues (toued_dbg_wgrad_visits);
* the recurrent backward's outputs DG (dr_pre, dz_pre, d(W_hn h + b_hn)) and dX3/dX4 on 192 sampled rows of the
  K*R = 163,840 (update, agent-worker) rows, each row's whole T-step sequence, against float64 autograd of the same
  GRU + heads on that row's saved inputs and head cotangents (relative L2 < 1e-5 per output; the relu decisions
  taken from the device, every differing one within 5e-6 of the kink, as test_gru_backward_matches_autograd).
"""
import math

import numpy as np
import pytest
import torch

from oracle import lpg as olpg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c2_step():
    from toued import _lib
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = parse_args(["--env_mode", "tabular", "--num_agents", "512", "--num_mini_batches", "1",
                       "--score_function", "random", "--seed", "11"])
    tr = Trainer(args)
    st = tr.step_fn
    assert (st.N, st.W, st.T, st.K) == (512, 64, 20, 5) and st.gru.M == 3_276_800 and st.gru.fused and st.gru.bfp
    tr.meta_step()                               # warm: plans, caches
    st.gru.keep_inputs = True                    # the backward's inputs, for the float64 VJP below
    visits = torch.zeros(4096, dtype=torch.int32, device="cuda")
    _lib.call("toued_dbg_wgrad_visits", _lib.ptr(visits), visits.numel())
    try:
        tr.meta_step()
        torch.cuda.synchronize()
    finally:
        _lib.lib().toued_dbg_wgrad_visits(None, 0)
    ntiles = int(_lib.lib().toued_dbg_wgrad_last_ntiles())
    return tr, visits, ntiles


def test_fullsize_wgrad_tiles_claimed_once(c2_step):
    _, visits, ntiles = c2_step
    v = visits.cpu().numpy()
    assert 64 <= ntiles <= 256
    assert (v[:ntiles] == 1).all(), np.nonzero(v[:ntiles] != 1)
    assert (v[ntiles:] == 0).all()


def test_fullsize_main_wgrad_matches_float64(c2_step):
    tr, _, _ = c2_step
    gru = tr.step_fn.gru
    F, M = gru.lay.F, gru.M
    ra = 256 + F + 1
    A = gru.a_rows()[:ra]                         # [h_in; x; 1]  [262][M] (rows of h_in's slab blocks)
    B = gru.dg_rows().reshape(3 * 256, M)         # [dr; dz; dhn] [768][M] (rows of the slab blocks)
    ref = torch.zeros(ra, 768, dtype=torch.float64, device="cuda")
    mag = torch.zeros_like(ref)
    step = 1 << 18
    for c0 in range(0, M, step):
        a = A[:, c0:c0 + step].double()
        b = B[:, c0:c0 + step].double()
        ref += a @ b.t()
        mag += a.abs() @ b.abs().t()
        del a, b
    G = gru.G.double()
    assert torch.isfinite(G).all()
    err = (G - ref).abs()
    tol = 2e-6 * math.sqrt(M) * mag + 1e-30
    assert (err <= tol).all(), float((err / tol).max())
    rel = float(torch.linalg.norm(G - ref) / torch.linalg.norm(ref))
    print(f"full-size main weight gradient: relative L2 {rel:.2e}, max err/bound {float((err / tol).max()):.2e}")
    assert rel < 1e-5, rel


def test_fullsize_backward_sampled_rows_match_float64(c2_step):
    tr, _, _ = c2_step
    st = tr.step_fn
    gru = st.gru
    K, T, R, W, F, M = st.K, st.T, st.R, st.W, gru.lay.F, gru.M
    done_all, eta, y_hat, d_pi_hat, d_y_hat = gru._last_bwd
    RH = gru.relu_out()                           # the device's relu decisions (the unfused kernel, same gate maths)
    torch.cuda.synchronize()
    rs = np.random.RandomState(5)
    rows = set(rs.choice(K * R, 186, replace=False).tolist()) | {0, R - 1, R, (K - 1) * R, K * R - 1, 7 * W + 63}
    rows = np.array(sorted(rows))
    ks, rr = rows // R, rows % R
    n = len(rows)
    tt = np.arange(T)
    cols = torch.from_numpy((ks[:, None] * T + tt[None, :]) * R + rr[:, None]).cuda()       # [n, T] column ids
    # inputs of the sampled rows, float64, [n, T, .]
    x = gru.A[256:256 + F][:, cols].permute(1, 2, 0).double().detach().requires_grad_(True)  # [n, T, F]
    a_idx, w_idx = torch.from_numpy(rr // W).cuda(), torch.from_numpy(rr % W).cuda()
    d = done_all[torch.from_numpy(ks).cuda()[:, None], a_idx[:, None], torch.arange(T, device="cuda")[None, :],
                 w_idx[:, None]].bool()                                                      # [n, T]
    mk = (RH[:, cols] > 0).permute(1, 2, 0)                                                  # [n, T, 256]
    dpi = d_pi_hat.view(K * T, R)[torch.from_numpy(ks * T).cuda()[:, None] + torch.arange(T, device="cuda")[None, :],
                                  torch.from_numpy(rr).cuda()[:, None]].double()            # [n, T]
    dy = d_y_hat.view(K * T, 8, R)[torch.from_numpy(ks * T).cuda()[:, None] + torch.arange(T, device="cuda")[None, :],
                                   :, torch.from_numpy(rr).cuda()[:, None]].double()        # [n, T, 8]
    flat = eta.double().detach().requires_grad_(True)
    P = olpg.unflatten(flat, F)
    h = torch.zeros(n, 256, dtype=torch.float64, device="cuda")
    pres, outs = [None] * T, [None] * T
    for t in reversed(range(T)):
        h = torch.where(d[:, t, None], torch.zeros_like(h), h)
        xt = x[:, t]
        rp = xt @ P["ir_w"] + P["ir_b"] + h @ P["hr_w"]
        zp = xt @ P["iz_w"] + P["iz_b"] + h @ P["hz_w"]
        hn = h @ P["hn_w"] + P["hn_b"]
        for v in (rp, zp, hn):
            v.retain_grad()
        rg, zg = torch.sigmoid(rp), torch.sigmoid(zp)
        ng = torch.tanh(xt @ P["in_w"] + P["in_b"] + rg * hn)
        h = (1 - zg) * ng + zg * h
        pres[t], outs[t] = (rp, zp, hn), h
    hst = torch.stack(outs, 1)                                                               # [n, T, 256]
    flips = hst.detach()[mk != (hst.detach() > 0)].abs()
    assert (flips < 5e-6).all(), flips.max()
    hs = torch.where(mk, hst, torch.zeros_like(hst))
    pi_ref = (hs @ P["pi_w"] + P["pi_b"])[..., 0]
    y_ref = torch.softmax(hs @ P["y_w"] + P["y_b"], -1)
    ((pi_ref * dpi).sum() + (y_ref * dy).sum()).backward()
    errs = {}
    DG = gru.dg_rows()
    for g, name in enumerate(("dr_pre", "dz_pre", "dhn")):
        ref = torch.stack([pres[t][g].grad for t in range(T)], 1)                            # [n, T, 256]
        got = DG[g][:, cols].permute(1, 2, 0).double()
        errs[name] = float(torch.linalg.norm(got - ref) / torch.linalg.norm(ref))
    for f, dX in ((3, gru.dX3), (4, gru.dX4)):
        got = dX.view(K * T, R)[torch.from_numpy(ks * T).cuda()[:, None] + torch.arange(T, device="cuda")[None, :],
                                torch.from_numpy(rr).cuda()[:, None]].double()
        ref = x.grad[..., f]
        errs[f"dX{f}"] = float(torch.linalg.norm(got - ref) / torch.linalg.norm(ref))
    print(f"full-size backward, {n} sampled rows: relative L2", {k: f"{v:.2e}" for k, v in errs.items()},
          f"relu decisions from the device differing from float64: {flips.numel()}")
    assert all(v < 1e-5 for v in errs.values()), errs
