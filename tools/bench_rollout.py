"""Micro-benchmark of the rollout kernel at the C2 shape (512 agents, tabular): the eval_agent rollout
(4 workers x episode length, returns only) and one training rollout (64 workers x T=20).

    python tools/bench_rollout.py [--iters 3]

Runs two warm-up meta-steps of the headline workload so the actor tables and levels are the ones the
bench sees, then times the kernels with HIP events on the launching stream.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    from toued.dist import init_from_env
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = parse_args(["--env_mode", "tabular", "--num_agents", "512", "--num_mini_batches", "1",
                       "--score_function", "random"])
    tr = Trainer(args, init_from_env())
    for _ in range(2):
        tr.meta_step()
    torch.cuda.synchronize()
    st = tr.step_fn
    ro, ag, K = st.ro, tr.agents, st.K

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return round(s.elapsed_time(e) / a.iters, 3)

    (_, _), ea_state = ro.batch_reset(st.keys_ea_reset, ag.levels, 4)
    res = {"eval_len": ro.eval_rollout_len}
    res["eval_rollout_ms"] = timed(lambda: st._eval_rollout(st.keys_ea_roll, st.theta_h[K], ag.levels, ea_state))
    state = ag.state.clone()
    res["train_rollout_ms"] = timed(lambda: ro.batch_rollout(st.keys_ea_roll, st.theta_h[K], ag.levels, state))
    ew = ea_state.shape[1] // ag.levels.shape[0]
    res["eval_draws_ms"] = timed(lambda: ro.eval_draws(st.keys_ea_roll, ag.levels, ew))
    draws = ro.eval_draws(st.keys_ea_roll, ag.levels, ew)
    res["eval_returns_from_draws_ms"] = timed(lambda: ro.eval_returns_from_draws(draws, st.theta_h[K], ag.levels,
                                                                                 ea_state))
    cum = st._eval_rollout(st.keys_ea_roll, st.theta_h[K], ag.levels, ea_state)
    cum3 = ro.eval_returns_from_draws(draws, st.theta_h[K], ag.levels, ea_state)
    res["three_launch_bit_identical"] = bool(torch.equal(cum, cum3))
    res["eval_mean_return"] = float(cum.mean())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
