"""Where two identical forwards' saves differ (unit, column, both values), for the det_fwd probe."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
import torch  # noqa: E402


def main():
    from toued.lpg import LPGGRU, LPGLayout, init_lpg_params, quad_blocks_to_rows
    N, K, W, T, F = 4, 2, 64, 20, 5
    R = N * W
    lay = LPGLayout(F)
    eta = init_lpg_params(0, F)
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn((F, K, T, R), generator=g, device="cuda")
    done = (torch.rand((K, N, T, W), generator=g, device="cuda") < 0.05).to(torch.uint8)
    res = []
    for rep in range(3):
        gru = LPGGRU(lay, R, T, K, W, "cuda")
        gru.pack(eta)
        gru.X.copy_(X)
        pi = torch.zeros(K, T, R, device="cuda")
        y = torch.zeros(K, T, 8, R, device="cuda")
        for k in range(K):
            gru.forward(k, gru.X, done[k], eta, pi, y)
        torch.cuda.synchronize()
        res.append({"h_in": gru.hin_rows().clone(), "r": gru.s_rows(0).clone(), "z": gru.s_rows(1).clone(),
                    "hn": gru.s_rows(3).clone(), "pi": pi.clone()})
    for n in res[0]:
        a, b, c = res[0][n], res[1][n], res[2][n]
        d = (a != b) | (a != c)
        print(n, "differs at", int(d.sum()), flush=True)
        if n in ("z", "h_in") and d.any():
            u, m = torch.nonzero(d, as_tuple=True)
            for i in range(min(12, u.numel())):
                uu, mm = int(u[i]), int(m[i])
                print(f"   unit {uu} col {mm} (row {mm % R} t {(mm // R) % T} k {mm // (T * R)}): {float(a[uu, mm]):.6f} "
                      f"{float(b[uu, mm]):.6f} {float(c[uu, mm]):.6f}  r {float(res[0]['r'][uu, mm]):.6f} "
                      f"hn {float(res[0]['hn'][uu, mm]):.6f}", flush=True)
            print("   units mod 4:", torch.bincount(u % 4).tolist(), " rows mod 32:", torch.bincount(m % 32, minlength=32).tolist())


if __name__ == "__main__":
    main()
