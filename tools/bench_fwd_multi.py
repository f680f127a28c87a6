"""C4's per-candidate LPG GRU forward (toued_gru_fwd_multi: 1024 candidates x 64 workers, T = 20, F = 7, no saves),
mean ms per launch over --iters launches after warmup (HIP events on the launching stream).

    python tools/bench_fwd_multi.py [--iters 10]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from toued import _lib as L
    from toued.lpg import LPGLayout, init_lpg_params
    N, W, T, F = 1024, 64, 20, 7
    R = N * W
    lay = LPGLayout(F)
    eta = init_lpg_params(0, F)
    g = torch.Generator(device="cuda").manual_seed(0)
    nd = lay.size
    x = (eta.reshape(1, nd) + 0.01 * torch.randn((N, nd), generator=g, device="cuda")).contiguous()
    fwdA = torch.zeros((N, L.lib().toued_gru_packed_floats(2)), device="cuda")
    X = torch.randn((F, T, R), generator=g, device="cuda")
    done = (torch.rand((N, T, W), generator=g, device="cuda") < 0.05).to(torch.uint8)
    pi_hat = torch.zeros(T, R, device="cuda")
    y_hat = torch.zeros(T, 8, R, device="cuda")
    st = L.stream_ptr()
    L.call("toued_gru_pack_fwd_multi", L.ptr(x), nd, N, lay.c_offsets, F, L.ptr(fwdA), st)

    def run():
        L.call("toued_gru_fwd_multi", R, T, W, F, W, L.ptr(X), T * R, 1, L.ptr(done), L.ptr(fwdA), L.ptr(x), nd,
               lay.c_offsets, L.ptr(pi_hat), L.ptr(y_hat), st)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        run()
    e.record()
    torch.cuda.synchronize()
    print(json.dumps({"gru_fwd_multi_ms": round(s.elapsed_time(e) / a.iters, 4)}), flush=True)


if __name__ == "__main__":
    main()
