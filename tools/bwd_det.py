"""Backward determinism / cross-kernel check (dev tool): runs toued_gru_bwd 3x on fixed inputs, reports
differences between repeats, and saves dX3/dX4/grad to gpurun_out/bwd_<tag>.pt for cross-kernel comparison."""
import os, sys, torch, numpy as np
sys.path.insert(0, "to-ued_amd")
from toued.lpg import LPGGRU, LPGLayout, init_lpg_params
N, W, T, K, F = 2, 64, 6, 2, 5
R = N * W
lay = LPGLayout(F)
torch.manual_seed(0)
eta = init_lpg_params(5, F)
eta += torch.randn_like(eta) * 0.05
gru = LPGGRU(lay, R, T, K, W, "cuda")
gru.pack(eta)
rs = np.random.RandomState(1)
gru.X.copy_(torch.from_numpy(rs.randn(F, K, T, R).astype(np.float32)))
done_t = torch.from_numpy((rs.rand(K, N, T, W) < 0.15).astype(np.uint8)).cuda()
pi_hat = torch.zeros(K, T, R, device="cuda"); y_hat = torch.zeros(K, T, 8, R, device="cuda")
for k in range(K):
    gru.forward(k, gru.X, done_t[k], eta, pi_hat, y_hat)
d_pi = torch.from_numpy(rs.randn(K, T, R).astype(np.float32)).cuda()
d_y = torch.from_numpy(rs.randn(K, T, 8, R).astype(np.float32)).cuda()
outs = []
for rep in range(3):
    gru.dX3.fill_(float("nan"))
    grad = torch.zeros(lay.size, device="cuda")
    gru.backward(done_t, eta, y_hat, d_pi, d_y, gru.X, grad)
    torch.cuda.synchronize()
    outs.append((gru.dX3.clone(), gru.dX4.clone(), gru.DG.clone(), grad.clone()))
    print("rep", rep, "nan in dX3:", int(torch.isnan(gru.dX3).sum()))
for i in (1, 2):
    print("rep", i, [float((a - b).abs().max()) for a, b in zip(outs[0], outs[i])])
tag = sys.argv[1] if len(sys.argv) > 1 else "x"
os.makedirs("gpurun_out", exist_ok=True)
torch.save({"dX3": outs[0][0].cpu(), "dX4": outs[0][1].cpu(), "grad": outs[0][3].cpu()}, f"gpurun_out/bwd_{tag}.pt")
