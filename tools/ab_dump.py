"""Bit-identity probe between two builds of the library: one meta-gradient step with fixed keys, every tensor the
step object holds (and the updated eta / agent tables) saved, then compared bit for bit across the two dumps.

    TOUED_LIB=<lib.so> python tools/ab_dump.py dump <out.pt> [mode] [N] [K]
    python tools/ab_dump.py compare <a.pt> <b.pt>
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402


def dump(out, mode="dense", N=64, K=5):
    from test_gpu_meta import _agents_for
    from toued.lpg import init_lpg_params
    from toued.meta import AdamState, LpgHyperparams, MetaGradStep
    W, T = 64, 20
    ro, ag = _agents_for(mode, N, W, T, 40)
    eta = init_lpg_params(71, 5)
    rng = torch.tensor([0, 123], dtype=torch.int32, device="cuda")
    st = MetaGradStep(ro, N, LpgHyperparams(num_agent_updates=K), False)
    res = {}
    for step in range(2):   # two steps: the second starts from the first's agents (history ring, adjoint reuse)
        m = st(rng + step, eta, AdamState(eta.numel(), "cuda"), ag)
        torch.cuda.synchronize()
        res[f"s{step}.return"] = m["lpg_agent_return"].clone()
    bufs = {}
    for k, v in vars(st).items():
        if torch.is_tensor(v):
            bufs[k] = v
        elif isinstance(v, (list, tuple)) and v and all(torch.is_tensor(x) for x in v):
            for i, x in enumerate(v):
                bufs[f"{k}[{i}]"] = x
    for k, v in vars(st.gru).items():
        if torch.is_tensor(v):
            bufs[f"gru.{k}"] = v
    bufs.update({"eta": eta, "theta": ag.theta, "phi": ag.phi, "state": ag.state, "step": ag.step})
    res.update({k: v.detach().cpu().clone() for k, v in bufs.items()})
    torch.save(res, out)
    print(f"dumped {len(res)} tensors to {out}", flush=True)


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = 0
    skip = ("wg_work", "work", "scratch", "embed_partial")   # scratch buffers whose stale parts are not results
    for k in A:
        if any(s in k for s in skip):
            continue
        x, y = A[k], B.get(k)
        if y is None or x.shape != y.shape:
            print(f"{k}: missing or shape differs", flush=True)
            bad += 1
            continue
        xb = x.view(torch.uint8) if x.is_floating_point() else x
        yb = y.view(torch.uint8) if y.is_floating_point() else y
        if not torch.equal(xb, yb):
            d = float((x.double() - y.double()).abs().nan_to_num(0).max()) if x.is_floating_point() else float("nan")
            print(f"{k}: DIFFERS max|diff| {d:.3e} n_diff {int((xb != yb).sum())} of {xb.numel()}", flush=True)
            bad += 1
    print(f"compared {len(A)} tensors: {'ALL BIT-IDENTICAL' if bad == 0 else f'{bad} differ'}", flush=True)
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        args = sys.argv[2:]
        dump(args[0], *(args[1:2]), *(int(x) for x in args[2:4]))
    else:
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
