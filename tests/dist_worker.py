"""Worker for the multi-rank tests (launched by tests/test_gpu_dist.py via torch.distributed.run).

Runs `--meta_steps` outer iterations of the training driver (toued.train.Trainer) with the
given reference flags on this rank's agent slice and saves what a single-process run must
reproduce: the LPG parameters (or the OpenES mean), and this rank's agents' levels/steps.
"""
from __future__ import annotations

import argparse
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--meta_steps", type=int, default=2)
    ap.add_argument("--es_updates", type=int, default=0)
    ap.add_argument("--max_lifetime", type=int, default=0)
    ap.add_argument("--force_term_odd", action="store_true",
                    help="finish with one more level_sampler.sample in which odd (global) agents are terminated")
    a, rest = ap.parse_known_args()
    from toued.dist import init_from_env
    from toued.parse_args import parse_args
    from toued.train import Trainer
    world = init_from_env()
    args = parse_args(rest)
    tr = Trainer(args, world)
    if a.max_lifetime:
        tr.sampler.max_lifetime = a.max_lifetime
    if args.use_es and a.es_updates:
        tr.step_fn.K = a.es_updates
    for _ in range(a.meta_steps):
        tr.meta_step()
    if a.force_term_odd:
        from toued import prng
        from toued.env import L_LIFETIME
        lo = 0 if tr.sl is None else tr.sl[0]
        gid = torch.arange(lo, lo + tr.agents.n, device=tr.agents.step.device)
        tr.agents.step = torch.where(gid % 2 == 1, tr.agents.levels[:, L_LIFETIME], tr.agents.step)
        ks = prng.split(tr.rng, 2)
        tr.buffer, tr.agents = tr.sampler.sample(ks[1].contiguous(), tr.buffer, tr.agents, tr.sl)
    torch.cuda.synchronize()
    res = {"levels": tr.agents.levels.cpu().numpy(), "step": tr.agents.step.cpu().numpy(),
           "theta": tr.agents.theta.cpu().numpy()}
    if args.use_es:
        res["mean"] = tr.step_fn.es.mean.cpu().numpy()
    else:
        res["eta"] = tr.eta.cpu().numpy()
    if tr.buffer is not None:
        res["buf_score"] = tr.buffer.score.cpu().numpy()
        res["buf_active"] = tr.buffer.active.cpu().numpy()
        res["buf_new"] = tr.buffer.new.cpu().numpy()
    np.savez(os.path.join(a.out, f"rank{world.rank}_of{world.size}.npz"), **res)
    if world.active:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
