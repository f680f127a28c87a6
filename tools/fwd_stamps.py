"""Per-phase timing of k_gru_fwd6<true> from in-kernel s_memtime stamps (a FWD_STAMPS=1 variant library):

    python tools/build_variant.py gru.hip FWD_STAMPS=1
    TOUED_LIB=to-ued_amd/exp/libtoued_FWD_STAMPS_1.so python tools/fwd_stamps.py

Runs the C2-shape forward (512 agents x 64 workers, T = 20; with --multi the C4 per-candidate forward: 1024
candidates x 64 workers, F = 7, no saves) and prints, for the first 64 workgroups, the mean shader-clock cycles of
each phase of a step: contraction issue (16 fp16 carry k-steps + the augmented k-step), the barrier behind it (MFMA
drain + wave skew), gate maths + saves + head partials, the head barrier, the head reduction + softmax tail; and the
whole step."""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
import torch  # noqa: E402


def main():
    from toued import _lib
    from toued.lpg import LPGGRU, LPGLayout, init_lpg_params
    multi = "--multi" in sys.argv
    N, W, T, K, F = (1024, 64, 20, 1, 7) if multi else (512, 64, 20, 1, 5)
    R = N * W
    lay = LPGLayout(F)
    eta = init_lpg_params(0, F)
    g = torch.Generator(device="cuda").manual_seed(0)
    if multi:
        L = _lib
        nd = lay.size
        x = (eta.reshape(1, nd) + 0.01 * torch.randn((N, nd), generator=g, device="cuda")).contiguous()
        fwdA = torch.zeros((N, L.lib().toued_gru_packed_floats(2)), device="cuda")
        X = torch.randn((F, T, R), generator=g, device="cuda")
        done = (torch.rand((N, T, W), generator=g, device="cuda") < 0.05).to(torch.uint8)
        pi_hat = torch.zeros(T, R, device="cuda")
        y_hat = torch.zeros(T, 8, R, device="cuda")
        st = L.stream_ptr()
        L.call("toued_gru_pack_fwd_multi", L.ptr(x), nd, N, lay.c_offsets, F, L.ptr(fwdA), st)
        for _ in range(3):
            L.call("toued_gru_fwd_multi", R, T, W, F, W, L.ptr(X), T * R, 1, L.ptr(done), L.ptr(fwdA), L.ptr(x), nd,
                   lay.c_offsets, L.ptr(pi_hat), L.ptr(y_hat), st)
    else:
        gru = LPGGRU(lay, R, T, K, W, "cuda")
        gru.pack(eta)
        gru.X.copy_(torch.randn(gru.X.shape, generator=g, device="cuda"))
        done = (torch.rand((K, N, T, W), generator=g, device="cuda") < 0.05).to(torch.uint8)
        pi_hat = torch.zeros(K, T, R, device="cuda")
        y_hat = torch.zeros(K, T, 8, R, device="cuda")
        for _ in range(3):
            gru.forward(0, gru.X, done[0], eta, pi_hat, y_hat)
    torch.cuda.synchronize()
    if "--pp" in sys.argv:
        # the ping-pong schedule (FWD_PP=1 FWD_STAMPS=1): per half, its three pieces of work and the barrier waits
        buf = np.zeros(64 * 32 * 2 * 6, np.uint64)
        fn = _lib.lib().toued_dbg_fwd_pp_stamps
        fn.argtypes = [ctypes.c_void_p]
        assert fn(buf.ctypes.data) == 0
        st = buf.reshape(64, 32, 2, 6)[:, 1:T - 1].astype(np.int64)   # steps 1 .. T-2 (both halves busy)
        names = {0: ["k 0-7", "k 8-15 + aug (+ heads)", "gate maths s"], 1: ["gate maths s-1", "k 0-7", "k 8-15 + aug"]}
        for grp in range(2):
            e = st[:, :, grp]
            work = [float((e[..., 2 * j + 1] - e[..., 2 * j]).mean()) for j in range(3)]
            wait = [float((e[..., 2 * j + 2] - e[..., 2 * j + 1]).mean()) for j in range(2)]
            step = float((e[:, 1:, 0] - e[:, :-1, 0]).mean())
            print(json.dumps({"half": grp, **{n: round(w) for n, w in zip(names[grp], work)},
                              "barrier waits (1st, 2nd)": [round(w) for w in wait], "step": round(step)}), flush=True)
        return
    buf = np.zeros(64 * 32 * 6, np.uint64)
    fn = _lib.lib().toued_dbg_fwd_stamps
    fn.argtypes = [ctypes.c_void_p]
    assert fn(buf.ctypes.data) == 0
    st = buf.reshape(64, 32, 6)[:, :T].astype(np.int64)
    ph = np.diff(st, axis=2)
    names = ["contraction issue", "barrier (MFMA drain)", "gate maths + saves + head partials", "head barrier",
             "head reduce + softmax"]
    res = {n: float(ph[:, :, i].mean()) for i, n in enumerate(names)}
    res["step total"] = float((st[:, 1:, 0] - st[:, :-1, 0]).mean())
    print(json.dumps({k: round(v) for k, v in res.items()}), flush=True)
    if "--gm" in sys.argv:   # inside the gate maths: done flags + gate_ain, row tile 0, row tile 1, to the barrier
        gb = np.zeros(64 * 32 * 4, np.uint64)
        fg = _lib.lib().toued_dbg_fwd_gm_stamps
        fg.argtypes = [ctypes.c_void_p]
        assert fg(gb.ctypes.data) == 0
        gm = gb.reshape(64, 32, 4)[:, :T].astype(np.int64)
        parts = {"done flags + gate_ain": gm[..., 0] - st[..., 2], "row tile 0": gm[..., 1] - gm[..., 0],
                 "row tile 1": gm[..., 2] - gm[..., 1], "head fold to barrier": st[..., 3] - gm[..., 2]}
        print(json.dumps({k: round(float(v.mean())) for k, v in parts.items()}), flush=True)


if __name__ == "__main__":
    main()
