"""The documented entry point ``python -m toued.train`` (README; the reference's train.py:14-82)
parses the reference's flags and runs, instead of importing the module and exiting 0."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "to-ued_amd")


def _run(*args, timeout=300):
    env = dict(os.environ, PYTHONPATH=PKG + os.pathsep + os.environ.get("PYTHONPATH", ""))
    return subprocess.run([sys.executable, "-m", "toued.train", *args], cwd=PKG, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_train_module_help_lists_reference_flags():
    r = _run("--help")
    assert r.returncode == 0, r.stderr
    for flag in ("--env_mode", "--num_agents", "--score_function", "--use_es", "--lifetime_conditioning",
                 "--num_mini_batches"):
        assert flag in r.stdout


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="checks the no-GPU failure path")
def test_train_module_runs_main_and_fails_loudly_without_gpu():
    """With no GPU the driver must reach Trainer and fail (the HIP path has no CPU fallback), not exit 0."""
    r = _run("--env_mode", "tabular", "--num_agents", "2", "--train_steps", "1")
    assert r.returncode != 0
