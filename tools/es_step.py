"""C4 ES steps (512 agents -> 1024 candidates, all_vrandlife, lifetime conditioning) for kernel traces:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/es -o run -- python3 tools/es_step.py 2

One warm-up step, then the given number of steps, each timed."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
import torch  # noqa: E402


def main():
    from toued.parse_args import parse_args
    from toued.train import Trainer
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    args = parse_args(["--env_mode", "all_vrandlife", "--num_agents", "512", "--num_mini_batches", "1", "--use_es",
                       "--lifetime_conditioning", "--lpg_learning_rate", "0.01"])
    tr = Trainer(args)
    for i in range(n + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.meta_step()
        torch.cuda.synchronize()
        print(f"step {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
