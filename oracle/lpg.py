"""torch-CPU (float64 by default) restatement of the LPG model — test oracle.

models/lpg.py:11-96 — ``LPG.__call__``: embedding MLP [16, 1] on y_t / y_tp1
(models/common.py:6-18), zeroed for y_tp1 where done; input
x = [r, d, pi, e(y_t), e(y_tp1) (, step, lifetime)]; reverse-time GRU with
done-reset (``LPGGRU``, flax 0.6.11 GRUCell: r/z sigmoid gates, n = tanh(W_in x
+ b_in + r*(W_hn h + b_hn)), h' = (1-z)*n + z*h; hidden width from the carry,
SURVEY §8c); heads pi_hat = Dense(1)(relu(h)), y_hat = softmax(Dense(8)(relu(h))).

Parameters are one flat vector in jax ``tree_flatten`` order of the flax param
dict (dict keys sorted; each leaf raveled row-major) — the same flat layout the
product uses (toued/lpg.py LPGLayout):
  Dense_0/{bias[1], kernel[H,1]}             pi head
  Dense_1/{bias[Y], kernel[H,Y]}             y head
  LPGGRU_0/GRUCell_0/hn/{bias[H], kernel[H,H]}, hr/kernel[H,H], hz/kernel[H,H],
                     in/{bias[H], kernel[F,H]}, ir/{bias, kernel}, iz/{bias, kernel}
  MLP_0/Dense_0/{bias[E], kernel[Y,E]}, MLP_0/Dense_1/{bias[1], kernel[E,1]}
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch


def layout(F: int, H: int = 256, Y: int = 8, E: int = 16):
    """OrderedDict name -> shape in flat order."""
    L = OrderedDict()
    L["pi_b"] = (1,)
    L["pi_w"] = (H, 1)
    L["y_b"] = (Y,)
    L["y_w"] = (H, Y)
    L["hn_b"] = (H,)
    L["hn_w"] = (H, H)
    L["hr_w"] = (H, H)
    L["hz_w"] = (H, H)
    L["in_b"] = (H,)
    L["in_w"] = (F, H)
    L["ir_b"] = (H,)
    L["ir_w"] = (F, H)
    L["iz_b"] = (H,)
    L["iz_w"] = (F, H)
    L["e1_b"] = (E,)
    L["e1_w"] = (Y, E)
    L["e2_b"] = (1,)
    L["e2_w"] = (E, 1)
    return L


def n_params(F: int, H: int = 256, Y: int = 8, E: int = 16) -> int:
    return int(sum(np.prod(s) for s in layout(F, H, Y, E).values()))


def unflatten(flat: torch.Tensor, F: int, H: int = 256, Y: int = 8, E: int = 16):
    out = {}
    off = 0
    for k, s in layout(F, H, Y, E).items():
        n = int(np.prod(s))
        out[k] = flat[off:off + n].reshape(s)
        off += n
    assert off == flat.numel()
    return out


def init_params(seed: int, F: int, H: int = 256, Y: int = 8, E: int = 16, dtype=np.float32) -> np.ndarray:
    """A flax-like initialisation (lecun-normal kernels, orthogonal recurrent kernels, zero biases).
    flax's exact init RNG derivation is not reproduced (parity unpinned)."""
    rs = np.random.RandomState(seed)
    parts = []
    for k, s in layout(F, H, Y, E).items():
        if k.endswith("_b"):
            parts.append(np.zeros(s))
        elif k in ("hn_w", "hr_w", "hz_w"):
            q, r = np.linalg.qr(rs.randn(H, H))
            parts.append(q * np.sign(np.diag(r))[None, :])
        else:
            fan_in = s[0]
            std = np.sqrt(1.0 / fan_in) / 0.87962566103423978
            parts.append(np.clip(rs.randn(*s), -2, 2) * std)
    return np.concatenate([p.ravel() for p in parts]).astype(dtype)


def embed(P, y):
    """MLP([16, 1]) (models/common.py:6-18): Dense(16) -> relu -> Dense(1)."""
    return torch.relu(y @ P["e1_w"] + P["e1_b"]) @ P["e2_w"] + P["e2_b"]


def lpg_apply(flat, r, d, pi, yt, yt1, step=None, lifetime=None, H: int = 256, Y: int = 8, E: int = 16,
              return_states=False, relu_mask=None, h_record=None):
    """models/lpg.py:48-85.  r,d,pi [B,T]; yt,yt1 [B,T,Y] -> pi_hat [B,T], y_hat [B,T,Y].

    step/lifetime: per-batch-row scalars [B] (raw values) when lifetime conditioning.
    relu_mask [B,T,H] (0/1), when given, replaces the ``h > 0`` decision of nn.relu(x) (models/lpg.py:81):
    a caller comparing with a float32 implementation takes its branch at outputs within rounding of the
    kink (the tests check that every disagreement sits there).  h_record (list) receives h_out [B,T,H].
    """
    F = 7 if step is not None else 5
    P = unflatten(flat, F, H, Y, E)
    df = d.to(flat.dtype)
    pyt = embed(P, yt)                                      # [B,T,1]
    pyt1 = embed(P, yt1)
    pyt1 = torch.where(d[..., None].bool(), torch.zeros_like(pyt1), pyt1)
    feats = [r[..., None], df[..., None], pi[..., None], pyt, pyt1]
    if step is not None:
        B, T = r.shape
        feats.append(step.to(flat.dtype)[:, None, None].expand(B, T, 1))
        feats.append(lifetime.to(flat.dtype)[:, None, None].expand(B, T, 1))
    x = torch.cat(feats, dim=-1)                            # [B,T,F]
    B, T, _ = x.shape
    h = torch.zeros(B, H, dtype=flat.dtype)
    outs = [None] * T
    states = {}
    for t in reversed(range(T)):
        h = torch.where(d[:, t, None].bool(), torch.zeros_like(h), h)
        xt = x[:, t]
        rg = torch.sigmoid(xt @ P["ir_w"] + P["ir_b"] + h @ P["hr_w"])
        zg = torch.sigmoid(xt @ P["iz_w"] + P["iz_b"] + h @ P["hz_w"])
        hn = h @ P["hn_w"] + P["hn_b"]
        ng = torch.tanh(xt @ P["in_w"] + P["in_b"] + rg * hn)
        if return_states:
            states[t] = (h, rg, zg, hn, ng)
        h = (1.0 - zg) * ng + zg * h
        outs[t] = h
    hs = torch.stack(outs, dim=1)                           # [B,T,H]
    if h_record is not None:
        h_record.append(hs.detach())
    a = torch.relu(hs) if relu_mask is None else hs * relu_mask.to(hs.dtype)
    pi_hat = (a @ P["pi_w"] + P["pi_b"])[..., 0]
    y_hat = torch.softmax(a @ P["y_w"] + P["y_b"], dim=-1)
    if return_states:
        return pi_hat, y_hat, hs, x, states
    return pi_hat, y_hat
