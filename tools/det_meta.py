"""Determinism probe of the meta-gradient step: two MetaGradStep instances on cloned agents and the same key, every
intermediate buffer compared bit for bit (first difference named), then the main reduction re-run on the second
instance's operands.

    python tools/det_meta.py [mode] [N] [K]
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402


def main():
    from test_gpu_meta import _agents_for, _clone_agents
    from toued.lpg import init_lpg_params
    from toued.meta import AdamState, LpgHyperparams, MetaGradStep
    mode = sys.argv[1] if len(sys.argv) > 1 else "dense"
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    W, T = 64, 20
    ro, ag0 = _agents_for(mode, N, W, T, 40)
    eta0 = init_lpg_params(71, 5)
    rng = torch.tensor([0, 123], dtype=torch.int32, device="cuda")
    steps = []
    for _ in range(2):
        ag = _clone_agents(ag0)
        eta = eta0.clone()
        st = MetaGradStep(ro, N, LpgHyperparams(num_agent_updates=K), False)
        st(rng, eta, AdamState(eta.numel(), "cuda"), ag)
        torch.cuda.synchronize()
        steps.append((st, eta))
    (a, ea), (b, eb) = steps
    ga, gb = a.gru, b.gru
    M = ga.M
    names = [("traj.obs_idx", a.traj.obs_idx, b.traj.obs_idx), ("X", ga.A[256:], gb.A[256:]),
             ("pi_hat", a.pi_hat, b.pi_hat), ("y_hat", a.y_hat, b.y_hat),
             ("h_in", ga.A[:256], gb.A[:256]), ("r", ga.S[0], gb.S[0]), ("z", ga.S[1], gb.S[1]),
             ("hn", ga.S[3], gb.S[3]), ("d_pi_hat", a.d_pi_hat, b.d_pi_hat), ("d_y_hat", a.d_y_hat, b.d_y_hat),
             ("DG", ga.DG, gb.DG), ("CE", ga.CE, gb.CE), ("dX3", ga.dX3, gb.dX3), ("GI", ga.GI, gb.GI),
             ("G", ga.G, gb.G), ("grad", a.grad, b.grad), ("eta", ea, eb)]
    for n, x, y in names:
        eq = torch.equal(x, y)
        d = "" if eq else f" max|diff| {float((x.double() - y.double()).abs().max()):.3e} n_diff {int((x != y).sum())}"
        print(f"{n:10s} {'same' if eq else 'DIFFERS'}{d}", flush=True)
    # the main reduction twice more on b's operands
    from toued import _lib
    F = ga.lay.F
    outs = []
    for _ in range(3):
        G = torch.full_like(gb.G, float("nan"))
        _lib.call("toued_wgrad_bfp_slab", 256 + F + 1, 768, M, _lib.ptr(gb.A), M, 256, _lib.ptr(gb.DG), M, 3,
                  _lib.ptr(gb.CE), _lib.ptr(G), _lib.ptr(gb.wg_work), gb.wg_work.numel(), _lib.stream_ptr())
        torch.cuda.synchronize()
        outs.append(G)
    print("wgrad reruns equal:", torch.equal(outs[0], outs[1]), torch.equal(outs[1], outs[2]),
          "equal to the step's G:", torch.equal(outs[0], gb.G), flush=True)


if __name__ == "__main__":
    main()
