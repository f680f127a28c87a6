"""GRU forward + backward against float64 autograd over many input seeds (dev tool, one process).

Separates an input-dependent precision failure from a timing hazard in the intermittent
test_gru_backward_matches_autograd[2-64-1.0-4.0] failure: the test's eta perturbation
was drawn from an unseeded generator when it failed, so every failing run had different inputs.  Here
each seed draws its own perturbation, inputs and cotangents; a seed whose relative L2 error exceeds the
test's 1e-5 is re-run --reruns times (bit-identical reruns = input-dependent) and localised: the first
(k, t, 64-row group) where dX3 or the gate cotangents DG leave 1e-4 of float64.
  gpurun -- timeout -k 10 300 python tools/gru_seed_sweep.py --seeds 200 --out gpurun_out/sweep.json"""
import argparse
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "to-ued_amd")
sys.path.insert(0, ".")
from toued.lpg import LPGGRU, LPGLayout, init_lpg_params  # noqa: E402
from oracle import lpg as olpg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seeds", type=int, default=200)
ap.add_argument("--seed0", type=int, default=0)
ap.add_argument("--wscales", default="4.0,1.0")
ap.add_argument("--N", type=int, default=2)
ap.add_argument("--reruns", type=int, default=3)
ap.add_argument("--only", default="", help="comma-separated seeds instead of the range")
ap.add_argument("--out", default="")
a = ap.parse_args()
N, W, T, K, F = a.N, 64, 6, 2, 5
R = N * W
M = K * T * R
lay = LPGLayout(F)
gru = LPGGRU(lay, R, T, K, W, "cuda", fused=False)   # DG[3] and RH are read below
eta0 = init_lpg_params(5, F)


def inputs(seed, wscale):
    g = torch.Generator(device="cpu").manual_seed(seed)
    eta = eta0.clone() + (torch.randn(eta0.shape, generator=g) * 0.05).cuda()
    for name in ("hr_w", "hz_w", "hn_w"):
        lay.view(eta, name).mul_(wscale)
    rs = np.random.RandomState(100000 + seed)
    xs = rs.randn(F, K, T, R).astype(np.float32)
    done = (rs.rand(K, N, T, W) < 0.15).astype(np.uint8)
    d_pi = rs.randn(K, T, R).astype(np.float32)
    d_y = rs.randn(K, T, 8, R).astype(np.float32)
    return eta, xs, done, d_pi, d_y


def run_device(eta, xs, done, d_pi, d_y):
    gru.pack(eta)
    gru.X.copy_(torch.from_numpy(xs))
    done_t = torch.from_numpy(done).cuda()
    pi_hat = torch.zeros(K, T, R, device="cuda")
    y_hat = torch.zeros(K, T, 8, R, device="cuda")
    for k in range(K):
        gru.forward(k, gru.X, done_t[k], eta, pi_hat, y_hat)
    grad = torch.zeros(lay.size, device="cuda")
    gru.backward(done_t, eta, y_hat, torch.from_numpy(d_pi).cuda(), torch.from_numpy(d_y).cuda(), gru.X, grad)
    torch.cuda.synchronize()
    return dict(grad=grad.cpu().double().numpy(), dX3=gru.dX3.cpu().double().numpy(),
                DG=gru.DG.cpu().double().numpy(), RH=gru.RH[:256].cpu().double().numpy())


def run_ref(eta, xs, done, d_pi, d_y, relu_mask=None):
    """float64 autograd; also the gate pre-activation cotangents dr, dz, d(W_hn h + b_hn), dn per (k, t) and
    h_out.  relu_mask (bool [256][M], the device's relu(h_out) > 0) replaces relu's own decision where given:
    the reference then differentiates the same branch of the kink as the device."""
    flat = torch.tensor(eta.cpu().numpy(), dtype=torch.float64, requires_grad=True)
    P = olpg.unflatten(flat, F)
    x = torch.tensor(xs, dtype=torch.float64, requires_grad=True)
    loss = 0.0
    keep = {}
    hins = {}
    hout = np.zeros((256, M))
    for k in range(K):
        xk = x[:, k].permute(2, 1, 0)
        d = torch.tensor(done[k].transpose(0, 2, 1).reshape(R, T).astype(bool))
        h = torch.zeros(R, 256, dtype=torch.float64)
        outs = [None] * T
        for t in reversed(range(T)):
            h = torch.where(d[:, t, None], torch.zeros_like(h), h)
            hins[k, t] = h.detach()
            xt = xk[:, t]
            rp = xt @ P["ir_w"] + P["ir_b"] + h @ P["hr_w"]
            zp = xt @ P["iz_w"] + P["iz_b"] + h @ P["hz_w"]
            hn = h @ P["hn_w"] + P["hn_b"]
            rg, zg = torch.sigmoid(rp), torch.sigmoid(zp)
            npre = xt @ P["in_w"] + P["in_b"] + rg * hn
            for nm, v in (("r", rp), ("z", zp), ("hn", hn), ("n", npre)):
                v.retain_grad()
                keep[nm, k, t] = v
            ng = torch.tanh(npre)
            h = (1 - zg) * ng + zg * h
            outs[t] = h
        hst = torch.stack(outs, 1)                                        # [R, T, 256]
        for t in range(T):
            c = (k * T + t) * R
            hout[:, c:c + R] = outs[t].detach().numpy().T
        if relu_mask is None:
            hs = torch.relu(hst)
        else:
            mk = np.stack([relu_mask[:, (k * T + t) * R:(k * T + t + 1) * R].T for t in range(T)], 1)
            hs = torch.where(torch.from_numpy(mk), hst, torch.zeros_like(hst))
        pi_ref = (hs @ P["pi_w"] + P["pi_b"])[..., 0]
        y_ref = torch.softmax(hs @ P["y_w"] + P["y_b"], -1)
        loss = loss + (pi_ref * torch.tensor(d_pi[k].T, dtype=torch.float64)).sum() + \
            (y_ref * torch.tensor(d_y[k].transpose(2, 0, 1), dtype=torch.float64)).sum()
    loss.backward()
    DG = np.zeros((4, 256, M))
    for gi, nm in enumerate(("r", "z", "hn", "n")):
        for k in range(K):
            for t in range(T):
                c = (k * T + t) * R
                DG[gi, :, c:c + R] = keep[nm, k, t].grad.numpy().T
    return dict(grad=flat.grad.numpy(), dX3=x.grad.numpy()[3], DG=DG, hout=hout)


def errors(dev, ref):
    e = {}
    for name in ("hr_w", "hz_w", "hn_w", "in_w", "pi_w", "y_w"):
        o = lay.offsets[name]
        sl = slice(o, o + int(np.prod(lay.shapes[name])))
        e[name] = float(np.linalg.norm(dev["grad"][sl] - ref["grad"][sl]) / max(np.linalg.norm(ref["grad"][sl]), 1e-300))
    e["dX3"] = float(np.linalg.norm(dev["dX3"] - ref["dX3"]) / np.linalg.norm(ref["dX3"]))
    return e


def localise(dev, ref):
    """first (k, t) in backward order (t ascending) and 64-row group whose DG slice or dX3 leaves 1e-4"""
    out = []
    for k in range(K):
        for t in range(T):
            c = (k * T + t) * R
            for grp in range(R // 64):
                cs = slice(c + 64 * grp, c + 64 * grp + 64)
                for gi, nm in enumerate(("dr", "dz", "dhn", "dn")):
                    a, b = dev["DG"][gi, :, cs], ref["DG"][gi, :, cs]
                    rel = float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))
                    if rel > 1e-4:
                        bad = np.abs(a - b) > 1e-4 * np.abs(b).max()
                        units, rows = np.nonzero(bad)
                        out.append(dict(k=k, t=t, group=grp, gate=nm, rel=rel, n_bad=int(bad.sum()),
                                        units=sorted(set(units.tolist()))[:16], rows=sorted(set(rows.tolist()))[:16]))
                        break
            if out:
                return out
    return out


ws = [float(s) for s in a.wscales.split(",")]
seeds = [int(x) for x in a.only.split(",")] if a.only else list(range(a.seed0, a.seed0 + a.seeds))
rec = {"seeds": seeds if a.only else a.seeds, "wscales": ws, "fail": [], "max_err": {}, "max_err_same_relu_branch": {}}
t0 = time.time()
for wscale in ws:
    worst = worst_k = 0.0
    for s in seeds:
        inp = inputs(s, wscale)
        dev = run_device(*inp)
        ref = run_ref(*inp)
        e = errors(dev, ref)
        m = max(e.values())
        worst = max(worst, m)
        worst_k = max(worst_k, max(errors(dev, run_ref(*inp, relu_mask=dev["RH"] > 0)).values()))
        if m >= 1e-5:
            reps = [run_device(*inp) for _ in range(a.reruns)]
            same = [all(np.array_equal(r[x], dev[x]) for x in ("grad", "dX3", "DG")) for r in reps]
            loc = localise(dev, ref)
            # relu kink: elements where the device's relu(h_out) > 0 decision differs from float64's
            flip = (dev["RH"] > 0) != (ref["hout"] > 0)
            fl = [dict(unit=int(u), col=int(c), k=int(c // (T * R)), t=int(c // R % T), row=int(c % R),
                       h_ref=float(ref["hout"][u, c]), relu_dev=float(dev["RH"][u, c])) for u, c in zip(*np.nonzero(flip))]
            e_kink = errors(dev, run_ref(*inp, relu_mask=dev["RH"] > 0))
            f = dict(seed=s, wscale=wscale, errs=e, reruns_bit_identical=same, first_bad=loc, relu_flips=fl[:8],
                     n_relu_flips=len(fl), errs_same_relu_branch=e_kink)
            rec["fail"].append(f)
            print("FAIL", json.dumps(f), flush=True)
        if s % 20 == 0:
            print(f"wscale {wscale} seed {s}: max rel err {m:.2e} (worst so far {worst:.2e}, same relu branch "
                  f"{worst_k:.2e}) {time.time() - t0:.0f} s", flush=True)
    rec["max_err"][str(wscale)] = worst
    rec["max_err_same_relu_branch"][str(wscale)] = worst_k
print(json.dumps({k: v for k, v in rec.items() if k != "fail"}), f"{len(rec['fail'])} failing seeds")
if a.out:
    with open(a.out, "w") as fh:
        json.dump(rec, fh, indent=1)
