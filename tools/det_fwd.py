"""Forward-save coverage probe: the split-precision forward at a given shape into saves pre-filled with NaN, twice;
reports per array how many elements stay unwritten and whether the two runs agree.

    python tools/det_fwd.py [N] [K]
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
import torch  # noqa: E402


def main():
    from toued.lpg import LPGGRU, LPGLayout, init_lpg_params, quad_blocks_to_rows
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    W, T, F = 64, 20, 5
    R = N * W
    lay = LPGLayout(F)
    eta = init_lpg_params(0, F)
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn((F, K, T, R), generator=g, device="cuda")
    done = (torch.rand((K, N, T, W), generator=g, device="cuda") < 0.05).to(torch.uint8)
    res = []
    for rep in range(2):
        gru = LPGGRU(lay, R, T, K, W, "cuda")
        gru.pack(eta)
        gru.A[:256].fill_(float("nan"))
        gru.S.fill_(float("nan"))
        gru.X.copy_(X)
        pi = torch.zeros(K, T, R, device="cuda")
        y = torch.zeros(K, T, 8, R, device="cuda")
        for k in range(K):
            gru.forward(k, gru.X, done[k], eta, pi, y)
        torch.cuda.synchronize()
        arrs = {"h_in": gru.A[:256].clone(), "r": gru.S[0].clone(), "z": gru.S[1].clone(), "hn": gru.S[3].clone()}
        for n, a in arrs.items():
            bad = torch.isnan(a)
            if bad.any():
                rows = quad_blocks_to_rows(bad.reshape(-1).float(), gru.M)
                u, m = torch.nonzero(rows, as_tuple=True)
                print(f"run {rep} {n}: {int(bad.sum())} unwritten; units {sorted(set(u.tolist()))[:16]} "
                      f"cols mod 32 {sorted(set((m % 32).tolist()))[:16]} cols {m[:8].tolist()}", flush=True)
            else:
                print(f"run {rep} {n}: all written", flush=True)
        res.append(arrs)
    for n in res[0]:
        print(n, "runs equal:", torch.equal(res[0][n], res[1][n]), flush=True)


if __name__ == "__main__":
    main()
