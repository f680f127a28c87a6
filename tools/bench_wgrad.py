"""Weight-gradient GEMM variants at the C2 shape: G[264, 768] = A[264, M] . DG[768, M]^T, M = 3.28M."""
import json
import os
import sys

import torch


def timed(fn, iters=3):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters, 3)


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 5 * 20 * 32768
    A = torch.randn(264, M, device="cuda")
    DG = torch.randn(4, 256, M, device="cuda")
    B = DG[0:3].reshape(768, M)
    res = {"M": M, "blas_pref": os.environ.get("TORCH_BLAS_PREFER_HIPBLASLT", "default")}
    res["mm_A_Bt"] = timed(lambda: torch.mm(A, B.t()))
    res["mm_B_At_T"] = timed(lambda: torch.mm(B, A.t()))
    K = 5
    Ak = A.view(264, K, M // K).permute(1, 0, 2)
    Bk = B.view(768, K, M // K).permute(1, 0, 2)
    res["bmm5_sum"] = timed(lambda: torch.bmm(Ak, Bk.transpose(1, 2)).sum(0))
    for ch in (8, 32):
        Ac = A.view(264, ch, M // ch).permute(1, 0, 2)
        Bc = B.view(768, ch, M // ch).permute(1, 0, 2)
        res[f"bmm{ch}_sum"] = timed(lambda: torch.bmm(Ac, Bc.transpose(1, 2)).sum(0))
    X6 = A[256:262]
    res["mm_Gn"] = timed(lambda: torch.mm(X6, DG[3].t()))
    RH = torch.randn(257, M, device="cuda")
    DH = torch.randn(9, M, device="cuda")
    res["mm_heads"] = timed(lambda: torch.mm(RH, DH.t()))
    flops = 2 * 264 * 768 * M
    res["tflops_mm_A_Bt"] = round(flops / (res["mm_A_Bt"] * 1e-3) / 1e12, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
