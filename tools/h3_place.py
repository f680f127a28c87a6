"""Where and when k_wgrad_h3's workgroups ran (an H3_PLACE=1 variant library), for the intermittent slow launches:

    python tools/build_variant.py wgrad.hip H3_PLACE=1
    TOUED_LIB=to-ued_amd/exp/libtoued_H3_PLACE_1.so python tools/h3_place.py [steps]

Runs C2 meta-steps (N=512 tabular) and prints per launch: the span, how many workgroups started late (> 50 us after
the first), the XCC of each workgroup against blockIdx % 8, and per-XCC workgroup counts."""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
import torch  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    from toued import _lib as L
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = parse_args(["--env_mode", "tabular", "--num_agents", "512", "--num_mini_batches", "1",
                       "--score_function", "random"])
    tr = Trainer(args)
    for _ in range(steps):
        tr.meta_step()
    torch.cuda.synchronize()
    buf = np.zeros(64 * 256 * 4, dtype=np.uint64)
    n = ctypes.c_uint(0)
    fn = L.lib().toued_dbg_h3_place
    fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint)]
    assert fn(buf.ctypes.data, ctypes.byref(n)) == 0
    buf = buf.reshape(64, 256, 4)
    ev = np.zeros(64 * 64 * 2, dtype=np.uint32)
    ne = ctypes.c_uint(0)
    fe = L.lib().toued_dbg_evr_place
    fe.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint)]
    assert fe(ev.ctypes.data, ctypes.byref(ne)) == 0
    ev = ev.reshape(64, 64, 2)
    print(f"eval_returns launches {ne.value}, h3 launches {n.value}")
    for li in range(min(n.value, 64)):
        e = buf[li]
        idx = np.nonzero(e[:, 2] > 0)[0]
        G = len(idx)
        st, en = e[idx, 2].astype(np.int64), e[idx, 3].astype(np.int64)
        t0 = st.min()
        late = int((st - t0 > 5000).sum())          # 100 MHz ticks: 50 us
        xcc = (e[idx, 0] & 0xF).astype(int)
        off = (xcc - idx) % 8
        se = ((e[idx, 1].astype(np.int64) >> 13) & 7).astype(int)
        lx = xcc[st - t0 > 5000]
        ls = se[st - t0 > 5000]
        rr = np.bincount(off, minlength=8)
        per = np.bincount(xcc, minlength=8)
        print(f"launch {li:2d}: {G} WGs span {(en.max() - t0) / 100:7.0f} us  late {late:3d}  "
              f"xcc-blockIdx offsets {rr.tolist()}  per-XCC {per.tolist()}  "
              f"late WG first start +{(np.sort(st - t0)[-1]) / 100:.0f} us  late on (xcc,se) {list(zip(lx.tolist(), ls.tolist()))}")
        tab = np.zeros((8, 4), int)
        for a_, b_ in zip(xcc, se):
            tab[a_, b_ & 3] += 1
        print("      tile WGs per (xcc, se):", tab.tolist())
        if li < ne.value:
            ex = ev[li, :8]
            print(f"      eval_returns blocks: XCC {[(int(x) & 15) for x in ex[:, 0]]}  "
                  f"CU {[((int(h) >> 8) & 15, (int(h) >> 13) & 7) for h in ex[:, 1]]}")


if __name__ == "__main__":
    main()
