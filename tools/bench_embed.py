"""Micro-benchmark of toued_embed_bwd (the embedding-MLP parameter gradient) at the C2 shape, on a real meta-step's
tensors (bench.py's Trainer: N=512 tabular, W=64, T=20, K=5), over a sweep of workgroup counts.

    python tools/bench_embed.py [--blocks 384,768,1536] [--iters 20]

Prints one JSON line per workgroup count: mean ms per launch (HIP events on the launching stream) and the
meta-gradient slice it produces, relative to the production count's (768)."""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", default="768,384,1024,1536,2048")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--save", default="", help="save the first count's gradient (float64) to this file")
    a = ap.parse_args()
    from toued import _lib as L
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = parse_args(["--env_mode", "tabular", "--num_agents", "512", "--num_mini_batches", "1",
                       "--score_function", "random"])
    tr = Trainer(args, None)
    for _ in range(2):
        tr.meta_step()
    torch.cuda.synchronize()
    s = tr.step_fn
    N, W, T, K, D, R = s.N, s.W, s.T, s.K, s.D, s.R
    e1w, e1b, e2w = s._eta(tr.eta, "e1_w"), s._eta(tr.eta, "e1_b"), s._eta(tr.eta, "e2_w")
    t = s.traj
    ref = None
    for nb in [int(x) for x in a.blocks.split(",")]:
        part = torch.zeros(nb, 161, device="cuda")

        def run():
            L.call("toued_embed_bwd", N, W, T, D, K, L.ptr(s._phi_store), s._phi_store[0].numel(), s._ring_last,
                   L.ptr(t.obs_idx),
                   t.obs_idx[0].numel(), L.ptr(t.obs_time), L.ptr(t.done), t.done[0].numel(), L.ptr(s.gru.dX3),
                   L.ptr(s.gru.dX4), T * R, L.ptr(e1w), L.ptr(e1b), L.ptr(e2w), L.ptr(part), nb, L.stream_ptr())
        run()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(a.iters):
            run()
        ev[1].record()
        torch.cuda.synchronize()
        g = part.double().sum(0)
        if ref is None:
            ref = g
        rel = float((g - ref).norm() / ref.norm())
        print(json.dumps({"blocks": nb, "embed_bwd_ms": round(ev[0].elapsed_time(ev[1]) / a.iters, 4),
                          "rel_vs_first": rel, "g_norm": float(g.norm()), "g_head": [float(x) for x in g[:3]]}),
              flush=True)
        if a.save and nb == int(a.blocks.split(",")[0]):
            torch.save(g.cpu(), a.save)


if __name__ == "__main__":
    main()
