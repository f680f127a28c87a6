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
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "to-ued_amd"))
    from toued import _lib as L
    C = torch.empty(262, 768, device="cuda")
    work = torch.empty(max(int(L.lib().toued_wgrad_workspace_floats(262, 768, M)),
                           int(L.lib().toued_wgrad_workspace_floats(6, 256, M)),
                           int(L.lib().toued_wgrad_workspace_floats(9, 257, M))), device="cuda")
    res["toued_wgrad"] = timed(lambda: L.call("toued_wgrad", 262, 768, M, L.ptr(A), M, L.ptr(B), M, L.ptr(C), L.ptr(work), work.numel(), L.stream_ptr()))
    A[:256].uniform_(-1, 1)
    CE = torch.full((M,), 0, dtype=torch.int8, device="cuda")      # columns of N(0,1) data: max < 8 -> 2^11
    CE.fill_(11)
    wb = torch.empty(int(L.lib().toued_wgrad_bfp_workspace_floats(262, 768, M)), device="cuda")
    res["toued_wgrad_bfp"] = timed(lambda: L.call("toued_wgrad_bfp", 262, 768, M, L.ptr(A), M, 256, L.ptr(B), M,
                                                  L.ptr(CE), L.ptr(C), L.ptr(wb), wb.numel(), L.stream_ptr()))
    ref = torch.mm(A[:262], B.t())
    res["bfp_max_rel_vs_mm"] = float(((C - ref).abs().max() / ref.abs().max()))
    L.call("toued_wgrad", 262, 768, M, L.ptr(A), M, L.ptr(B), M, L.ptr(C), L.ptr(work), work.numel(), L.stream_ptr())
    res["max_rel_vs_mm"] = float(((C - ref).abs().max() / ref.abs().max()))
    X6 = A[256:262]
    res["mm_Gn"] = timed(lambda: torch.mm(X6, DG[3].t()))
    Cn = torch.empty(6, 256, device="cuda")
    res["toued_Gn"] = timed(lambda: L.call("toued_wgrad", 6, 256, M, L.ptr(A) + 4 * 256 * M, M, L.ptr(DG[3]), M,
                                           L.ptr(Cn), L.ptr(work), work.numel(), L.stream_ptr()))
    RH = torch.randn(257, M, device="cuda")
    DH = torch.randn(9, M, device="cuda")
    res["mm_heads"] = timed(lambda: torch.mm(RH, DH.t()))
    Ch = torch.empty(9, 257, device="cuda")
    res["toued_heads"] = timed(lambda: L.call("toued_wgrad", 9, 257, M, L.ptr(DH), M, L.ptr(RH), M, L.ptr(Ch),
                                              L.ptr(work), work.numel(), L.stream_ptr()))
    flops = 2 * 264 * 768 * M
    res["tflops_mm_A_Bt"] = round(flops / (res["mm_A_Bt"] * 1e-3) / 1e12, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
