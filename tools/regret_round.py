"""C3 regret rounds (512 antagonists, all_shortlife) for kernel traces:

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rr -o run -- python3 tools/regret_round.py 3

Runs one warm-up round and then the given number of rounds (every agent terminated, so every level is scored)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
import torch  # noqa: E402


def main():
    from toued.env import L_LIFETIME
    from toued.parse_args import parse_args
    from toued.train import Trainer
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    args = parse_args(["--env_mode", "all_shortlife", "--num_agents", "512", "--num_mini_batches", "1",
                       "--score_function", "alg_regret"])
    tr = Trainer(args)
    for i in range(n + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.agents.step = tr.agents.levels[:, L_LIFETIME].clone()
        tr.buffer, tr.agents = tr.sampler.sample(tr.rng, tr.buffer, tr.agents)
        torch.cuda.synchronize()
        print(f"round {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
