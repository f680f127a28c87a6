"""bench.py --gpus N starts its own N ranks (torch.distributed.run child) — CPU/gloo, world size 2.

The driver runs `python bench.py --gpus N` as well as the torchrun form; both must produce one JSON
line from rank 0 with n_gpus = N, and asking for more GPUs than the node has must fail loudly.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _env():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    return env


@pytest.mark.parametrize("n", [2, 8])
def test_bench_self_launches_ranks(n):
    """n = 8 is the driver's C5 node: eight gloo ranks through the same launcher, barrier and MAX timing."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--launcher_selftest"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["ranks_seen"] == n
    # max over ranks: rank r sleeps 10 (r + 1) ms inside the timed region
    assert out["max_dt"] >= 0.01 * n
    assert out["sum_ranks"] == n * (n + 1) / 2
    assert out["slice0"] == [0, 4096 // n, 4096] and out["gathered_ok"]


def test_bench_too_many_gpus_fails_loudly():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode != 0
    assert "requested but this node has" in (r.stderr + r.stdout)


def test_bench_world_size_mismatch_fails():
    env = _env()
    env.update(WORLD_SIZE="3", RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], capture_output=True, text=True,
                       timeout=240, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=3" in (r.stderr + r.stdout)
