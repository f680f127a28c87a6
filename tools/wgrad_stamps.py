"""Per-slab timing of k_wgrad_h3 from in-kernel s_memtime stamps (a WG_STAMPS=1 variant library):

    python tools/build_variant.py wgrad.hip WG_STAMPS=1
    TOUED_LIB=to-ued_amd/exp/libtoued_WG_STAMPS_1.so python tools/wgrad_stamps.py

Runs the C2-shape reduction (tools/bench_wgrad.py's operands) and prints the mean shader cycles per slab of: tiles
0-7, tiles 8-16 (with the A-slab LDS writes), the barrier, and the slab total, over the first 64 workgroups' waves."""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
import torch  # noqa: E402


def main():
    from toued import _lib as L
    M = 5 * 20 * 32768
    A = torch.randn(264, M, device="cuda")
    A[:256].uniform_(-1, 1)
    B = torch.randn(768, M, device="cuda")
    CE = torch.full((M,), 11, dtype=torch.int8, device="cuda")
    C = torch.empty(262, 768, device="cuda")
    wb = torch.empty(int(L.lib().toued_wgrad_bfp_workspace_floats(262, 768, M)), device="cuda")
    for _ in range(2):
        L.call("toued_wgrad_bfp", 262, 768, M, L.ptr(A), M, 256, L.ptr(B), M, L.ptr(CE), L.ptr(C), L.ptr(wb),
               wb.numel(), L.stream_ptr())
    torch.cuda.synchronize()
    buf = np.zeros(64 * 8 * 64 * 4, np.uint64)
    fn = L.lib().toued_dbg_wgrad_stamps
    fn.argtypes = [ctypes.c_void_p]
    assert fn(buf.ctypes.data) == 0
    st = buf.reshape(64, 8, 64, 4).astype(np.int64)
    nw = 8 if st[:, 4:].any() else 4                  # k_wgrad_h3<8, 2> (default) or <4, 3> (TOUED_WGRAD_NW4=1)
    st = st[:, :nw, 1:63]
    mfma = 17 * (2 if nw == 8 else 3) * 3               # MFMAs per wave and slab
    res = {"waves": nw, "tiles 0-7": float((st[..., 1] - st[..., 0]).mean()),
           "tiles 8-16": float((st[..., 2] - st[..., 1]).mean()),
           "barrier": float((st[..., 3] - st[..., 2]).mean()),
           "slab": float((st[:, :, 1:, 0] - st[:, :, :-1, 0]).mean()),
           "ideal MFMA issue per SIMD (x 16 cycles)": mfma * 16 * nw // 4}
    print(json.dumps({k: round(v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
