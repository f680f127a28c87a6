"""Micro-benchmark of the LPG GRU kernels at the C2 shape (N=512 agents x W=64, T=20, K=5).

    python tools/bench_gru.py [--iters 3] [--which fwd|bwd|both]

Times toued_gru_fwd (one launch per inner update) and toued_gru_bwd (one launch over all K)
with HIP events on the launching stream; prints ms and TFLOP/s.  Used for kernel work and for
focused rocprofv3 PMC passes (tools/profile.sh runs the whole bench instead).
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--which", default="both")
    ap.add_argument("--agents", type=int, default=512)
    a = ap.parse_args()
    from toued.lpg import LPGGRU, LPGLayout, init_lpg_params
    N, W, T, K, F = a.agents, 64, 20, 5, 5
    R = N * W
    lay = LPGLayout(F)
    eta = init_lpg_params(0, F)
    gru = LPGGRU(lay, R, T, K, W, "cuda")
    gru.pack(eta)
    g = torch.Generator(device="cuda").manual_seed(0)
    gru.X.copy_(torch.randn(gru.X.shape, generator=g, device="cuda"))
    done = (torch.rand((K, N, T, W), generator=g, device="cuda") < 0.05).to(torch.uint8)
    pi_hat = torch.zeros(K, T, R, device="cuda")
    y_hat = torch.zeros(K, T, 8, R, device="cuda")
    d_pi = torch.randn(K, T, R, generator=g, device="cuda") * 1e-3
    d_y = torch.randn(K, T, 8, R, generator=g, device="cuda") * 1e-3
    res = {}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.iters

    def fwd():
        for k in range(K):
            gru.forward(k, gru.X, done[k], eta, pi_hat, y_hat)

    if a.which in ("fwd", "both"):
        ms = timed(fwd) / K
        res["gru_fwd_ms"] = round(ms, 3)
        res["gru_fwd_tflops"] = round(R * T * 406080 / (ms * 1e-3) / 1e12, 1)
    else:
        fwd()
    if a.which in ("bwd", "both"):
        from toued import _lib
        L = _lib
        o = gru

        def bwd():
            if o.fused:   # the recurrent backward with both small weight-gradient products (and their reduction)
                L.call("toued_gru_bwd_fused", R, T, W, K, L.ptr(done), done[0].numel(), L.ptr(o.bwdA), L.ptr(eta),
                       lay.c_offsets, L.ptr(y_hat), L.ptr(d_pi), L.ptr(d_y), L.ptr(o.A), L.ptr(o.S[0]),
                       L.ptr(o.S[1]), L.ptr(o.S[3]), o.M, L.ptr(o.DG), L.ptr(o.dX3), L.ptr(o.dX4), L.ptr(o.CE),
                       L.ptr(o.GI), L.ptr(o.wg_work), o.wg_work.numel(), L.stream_ptr())
                return
            L.call("toued_gru_bwd", R, T, W, K, L.ptr(done), done[0].numel(), L.ptr(o.bwdA), L.ptr(eta),
                   lay.c_offsets, L.ptr(y_hat), L.ptr(d_pi), L.ptr(d_y), L.ptr(o.A), L.ptr(o.S[0]), L.ptr(o.S[1]),
                   L.ptr(o.S[2]), L.ptr(o.S[3]), o.M, L.ptr(o.DG), L.ptr(o.RH), L.ptr(o.DH), L.ptr(o.dX3),
                   L.ptr(o.dX4), L.ptr(o.CE) if o.bfp else None, L.stream_ptr())
        ms = timed(bwd)
        res["gru_bwd_ms"] = round(ms, 3)
        res["gru_bwd_fused_small"] = bool(o.fused)
        res["gru_bwd_tflops"] = round(K * R * T * 393216 / (ms * 1e-3) / 1e12, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
