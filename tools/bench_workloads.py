"""Secondary workloads of BASELINE.json (not the headline line, which is bench.py / C2).

    python tools/bench_workloads.py --workload groove [--steps 2] [--warmup 1] [--agents 512]
    python tools/bench_workloads.py --workload es     [--steps 1] [--warmup 1] [--agents 512]

groove (C3): --score_function alg_regret --env_mode all_shortlife, N agents.  Times
  (a) the LPG meta-gradient step (K=5), and
  (b) LevelSampler.sample with every agent terminated: _reset_lowest_scoring, one A2C
      antagonist per agent trained for max_lifetime=250 updates (W=64, T=20), two 64-worker
      eval_agent rollouts per agent, the buffer update and the replay/random selection.
  The reference scores every agent on every meta-step (level_sampler.py:176-181) and keeps
  only the terminated agents' scores; this build scores only terminated agents, so (b) is
  exactly its per-meta-step regret cost and (a)+(b) the reference-equivalent meta-step.
es (C4): --use_es --lifetime_conditioning --env_mode all_vrandlife, N agents -> 2N candidates,
  each trained with its own LPG for max_lifetime=250 updates, then fitness + OpenES tell.

Prints one JSON line per workload with agent-env-steps/sec (train rollouts only) and the
per-phase times.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))

import torch  # noqa: E402


def _sync_time(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n, out


def groove(a):
    from toued.env import L_LIFETIME
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = parse_args(["--env_mode", "all_shortlife", "--num_agents", str(a.agents), "--num_mini_batches", "1",
                       "--score_function", "alg_regret"])
    tr = Trainer(args)
    W, T, K = args.env_workers, args.train_rollout_len, args.num_agent_updates
    N = a.agents
    for _ in range(a.warmup):
        tr.meta_step()
    t_meta, _ = _sync_time(lambda: tr.step_fn(tr.rng, tr.eta, tr.adam, tr.agents), a.steps)

    def regret_round():
        tr.agents.step = tr.agents.levels[:, L_LIFETIME].clone()
        tr.buffer, tr.agents = tr.sampler.sample(tr.rng, tr.buffer, tr.agents)
    regret_round()   # warm (graph capture)
    t_regret, _ = _sync_time(regret_round, a.steps)
    U = tr.sampler.max_lifetime
    a2c_steps = N * U * W * T
    meta_steps = N * W * T * K
    out = {"workload": "C3 GROOVE alg_regret env_mode=all_shortlife", "num_agents": N,
           "meta_step_ms": round(t_meta * 1e3, 2), "regret_sample_ms": round(t_regret * 1e3, 2),
           "a2c_agent_env_steps_per_sec": round(a2c_steps / t_regret, 1),
           "reference_equivalent_meta_step_ms": round((t_meta + t_regret) * 1e3, 2),
           "agent_env_steps_per_sec_reference_equivalent": round((meta_steps + a2c_steps) / (t_meta + t_regret), 1),
           "amortized_meta_step_ms (regret every lifetime/K meta-steps)":
               round((t_meta + t_regret * K / U) * 1e3, 2)}
    print(json.dumps(out), flush=True)


def es(a):
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = parse_args(["--env_mode", "all_vrandlife", "--num_agents", str(a.agents), "--num_mini_batches", "1",
                       "--use_es", "--lifetime_conditioning", "--lpg_learning_rate", "0.01"])
    tr = Trainer(args)
    W, T = args.env_workers, args.train_rollout_len
    K = tr.step_fn.K
    C = 2 * a.agents
    for _ in range(a.warmup):
        tr.meta_step()
    t, m = _sync_time(tr.meta_step, a.steps)
    steps = C * K * W * T
    out = {"workload": "C4 TA-LPG OpenES env_mode=all_vrandlife lifetime_conditioning", "num_agents": a.agents,
           "candidates": C, "updates_per_candidate": K, "es_step_ms": round(t * 1e3, 1),
           "agent_env_steps_per_sec": round(steps / t, 1),
           "gru_fwd_tflop_per_es_step": round(C * W * T * K * 409152 / 1e12, 1),
           "fitness_mean": float(m["fitness"]["mean"])}
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["groove", "es"], required=True)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--agents", type=int, default=512)
    a = ap.parse_args()
    {"groove": groove, "es": es}[a.workload](a)


if __name__ == "__main__":
    main()
