"""Accuracy of the LPG GRU forward against float64 (the f32-accuracy check of the bf16-split kernels).

    python tools/gru_accuracy.py            # default kernels
    TOUED_GRU_F32=1 python tools/gru_accuracy.py   # the f32-MFMA kernel, for comparison

Prints the max abs error of pi_hat, y_hat and the saved activations over T=20 steps of 4 agents x 64 workers
on random inputs (same construction as tests/test_gpu_meta.py::test_gru_forward_matches_oracle)."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from oracle import lpg as olpg
    from toued.lpg import LPGGRU, LPGLayout, init_lpg_params
    N, W, T, K = 4, 64, 20, 1
    R = N * W
    lay = LPGLayout(5)
    eta = init_lpg_params(3, 5)
    eta += torch.randn_like(eta) * 0.05
    gru = LPGGRU(lay, R, T, K, W, "cuda")
    gru.pack(eta)
    rs = np.random.RandomState(0)
    X = gru.X
    X.copy_(torch.from_numpy(rs.randn(5, K, T, R).astype(np.float32)))
    done = (rs.rand(K, N, T, W) < 0.1).astype(np.uint8)
    pi_hat = torch.zeros(K, T, R, device="cuda")
    y_hat = torch.zeros(K, T, 8, R, device="cuda")
    gru.forward(0, X, torch.from_numpy(done[0]).cuda(), eta, pi_hat, y_hat)
    torch.cuda.synchronize()
    P = olpg.unflatten(torch.tensor(eta.cpu().numpy(), dtype=torch.float64), 5)
    x = torch.tensor(X[:, 0].cpu().numpy(), dtype=torch.float64).permute(2, 1, 0)
    d = torch.tensor(done[0].transpose(0, 2, 1).reshape(R, T).astype(bool))
    h = torch.zeros(R, 256, dtype=torch.float64)
    outs, hins = [None] * T, [None] * T
    for t in reversed(range(T)):
        h = torch.where(d[:, t, None], torch.zeros_like(h), h)
        xt = x[:, t]
        rg = torch.sigmoid(xt @ P["ir_w"] + P["ir_b"] + h @ P["hr_w"])
        zg = torch.sigmoid(xt @ P["iz_w"] + P["iz_b"] + h @ P["hz_w"])
        ng = torch.tanh(xt @ P["in_w"] + P["in_b"] + rg * (h @ P["hn_w"] + P["hn_b"]))
        hins[t] = h
        h = (1 - zg) * ng + zg * h
        outs[t] = h
    hs = torch.relu(torch.stack(outs, 1))
    pi_ref = (hs @ P["pi_w"] + P["pi_b"])[..., 0].numpy()
    y_ref = torch.softmax(hs @ P["y_w"] + P["y_b"], -1).numpy()
    hin_gpu = gru.hin_rows().cpu().numpy().reshape(256, T, R).transpose(2, 1, 0)
    hin_ref = torch.stack(hins, 1).numpy()
    res = {"kernel": "f32" if os.environ.get("TOUED_GRU_F32") == "1" else "default",
           "pi_hat_max_abs": float(np.abs(pi_hat[0].cpu().numpy().T - pi_ref).max()),
           "y_hat_max_abs": float(np.abs(y_hat[0].cpu().numpy().transpose(2, 0, 1) - y_ref).max()),
           "h_in_max_abs": float(np.abs(hin_gpu - hin_ref).max()),
           "pi_hat_scale": float(np.abs(pi_ref).max())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
