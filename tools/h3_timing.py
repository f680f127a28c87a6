"""k_wgrad_h3 launch durations of C2 meta-steps with the step's kernel timers on or off (rocprofv3 kernel trace):
    rocprofv3 --kernel-trace --output-format csv -d DIR -- python3 tools/h3_timing.py STEPS TIMERS(0|1)
    python3 tools/h3_launches.py DIR"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
import torch  # noqa: E402


def main():
    steps, timers = int(sys.argv[1]), sys.argv[2] == "1"
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = parse_args(["--env_mode", "tabular", "--num_agents", "512", "--num_mini_batches", "1",
                       "--score_function", "random"])
    tr = Trainer(args)
    tr.meta_step()
    tr.step_fn.timers.enabled = timers
    for _ in range(steps):
        tr.meta_step()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
