"""Per-phase timing of k_gru_bwd6n from in-kernel s_memtime stamps (a BWD_STAMPS=1 variant library):

    python tools/build_variant.py gru.hip BWD_STAMPS=1
    TOUED_LIB=to-ued_amd/exp/libtoued_BWD_STAMPS_1.so python tools/bwd_stamps.py

Runs the C2-shape backward (tools/bench_gru.py's setup) and prints, for the first 64 workgroups, the mean shader
cycles of each phase of a step: head cotangents + barrier, memory part, row-max barrier, dr split + barriers, the
three gate contractions, and the step tail."""
import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
sys.path.insert(0, str(ROOT / "tools"))
import torch  # noqa: E402


def main():
    import bench_gru
    bench_gru_main = getattr(bench_gru, "setup", None)
    from toued import _lib
    from toued.lpg import LPGGRU, LPGLayout, init_lpg_params
    N, W, T, K, F = 512, 64, 20, 5, 5
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
    for k in range(K):
        gru.forward(k, gru.X, done[k], eta, pi_hat, y_hat)
    d_pi = torch.randn(K, T, R, device="cuda", generator=g) * 1e-3
    d_y = torch.randn(K, T, 8, R, device="cuda", generator=g) * 1e-3
    grad = torch.zeros(lay.size, device="cuda")
    for _ in range(2):
        gru.backward(done, eta, y_hat, d_pi, d_y, gru.X, grad)
    torch.cuda.synchronize()
    buf = np.zeros(64 * 32 * 8, np.uint64)
    fn = _lib.lib().toued_dbg_bwd_stamps
    fn.argtypes = [ctypes.c_void_p]
    assert fn(buf.ctypes.data) == 0
    st = buf.reshape(64, 32, 8)[:, :T].astype(np.int64)
    ph = np.diff(st, axis=2)                                  # 7 intra-step phases
    tail = st[:, 1:, 0] - st[:, :-1, 7]                       # step end -> next step start
    names = ["head+sync", "memory part", "rowmax sync", "dr split+syncs", "contract dr", "contract dz", "contract dhn"]
    res = {n: float(ph[:, :, i].mean()) for i, n in enumerate(names)}
    res["tail (dx, carry, sync)"] = float(tail.mean())
    res["step total"] = float((st[:, 1:, 0] - st[:, :-1, 0]).mean())
    print(json.dumps({k: round(v) for k, v in res.items()}), flush=True)
    # per-wave memory parts (BWD_WSTAMP): when each wave starts and ends its memory part relative to the workgroup's
    # first start, by wave and by its SIMD, and how long the last wave trails the first
    wf = getattr(_lib.lib(), "toued_dbg_bwd_wstamps", None)
    if wf is not None:
        wf.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        NWS = 8
        wb = np.zeros(64 * 32 * 8 * NWS, np.uint64)
        simd = np.zeros(64 * 8, np.int32)
        assert wf(wb.ctypes.data, simd.ctypes.data) == 0
        w = wb.reshape(64, 32, 8, NWS)[:, :T].astype(np.int64)
        t0 = w[:, :, :, 0].min(axis=2, keepdims=True)
        # the other per-wave points relative to the same origin: 2 pass dr start (after the dr split), 3 its last
        # MFMA issued, 4 after the barrier behind it, 5 pass dz start (refill + barrier done), 6 its last MFMA, 7 barrier
        names = {2: "pass_dr_start", 3: "pass_dr_issued", 4: "pass_dr_barrier", 5: "pass_dz_start",
                 6: "pass_dz_issued", 7: "pass_dz_barrier"}
        pts = {nm: (w[:, :, :, i] - t0[:, :, :]).mean(axis=(0, 1)).round().tolist() for i, nm in names.items()}
        print(json.dumps(pts), flush=True)
        start, end = w[:, :, :, 0] - t0, w[:, :, :, 1] - t0
        dur = end - start
        simd = simd.reshape(64, 8)
        out = {"wave_start_mean": start.mean(axis=(0, 1)).round().tolist(),
               "wave_end_mean": end.mean(axis=(0, 1)).round().tolist(),
               "wave_dur_mean": dur.mean(axis=(0, 1)).round().tolist(),
               "end_spread_mean (last - first wave)": float((end.max(axis=2) - end.min(axis=2)).mean()),
               "simd_of_wave (wg 0..3)": simd[:4].tolist()}
        # rank of each wave's end among the two waves on its SIMD: does the later one trail by the shared VALU?
        pair_gap = []
        for b_ in range(64):
            for sm in range(4):
                ws = np.nonzero(simd[b_] == sm)[0]
                if len(ws) == 2:
                    pair_gap.append(np.abs(end[b_, :, ws[0]] - end[b_, :, ws[1]]).mean())
        out["same_simd_end_gap_mean"] = float(np.mean(pair_gap)) if pair_gap else None
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
