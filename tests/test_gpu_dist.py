"""Data-parallel sharding of the agent axis on real kernels: two ranks sharing the
box's GPU (gloo collectives staged through the host) must reproduce a single-process run.

  * levels / agent steps per agent: bit-exact (every rank derives all N keys and keeps its slice)
  * LPG parameters after the meta-gradient all-reduce + Adam: within 1e-6 (float32 summation
    order of the gradient differs between one and two partial sums); agent actors after the second
    step (trained under those parameters, lr 40): within 1e-5 absolute
  * alg_regret buffer (replicated, updated from all-gathered scores): flags bit-exact, scores
    within 1e-6 — the regret of an agent depends only on its own key, level and actor
  * OpenES mean after the tell all-reduce: within 1e-6
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(nproc, out, flags):
    env = dict(os.environ, TOUED_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "tests" / "dist_worker.py"),
           "--out", str(out)] + flags
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return [dict(np.load(out / f"rank{i}_of{nproc}.npz")) for i in range(nproc)]


CASES = {
    "meta_grad": ["--env_mode", "dense", "--num_agents", "4", "--num_mini_batches", "1", "--num_agent_updates", "2",
                  "--score_function", "random"],
    "alg_regret": ["--env_mode", "mazes", "--num_agents", "4", "--num_mini_batches", "1", "--num_agent_updates",
                   "2", "--score_function", "alg_regret", "--buffer_size", "32", "--max_lifetime", "2",
                   "--force_term_odd"],
    "es": ["--env_mode", "all_vrandlife", "--num_agents", "4", "--num_mini_batches", "1", "--use_es",
           "--lifetime_conditioning", "--lpg_learning_rate", "0.01", "--es_updates", "2"],
}


@pytest.mark.parametrize("case", list(CASES))
def test_two_ranks_match_one(tmp_path, case):
    flags = CASES[case]
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    one = _run(1, tmp_path / "a", flags)[0]
    two = _run(2, tmp_path / "b", flags)
    for k in ("levels", "step"):
        assert np.array_equal(np.concatenate([t[k] for t in two]), one[k]), k
    np.testing.assert_allclose(np.concatenate([t["theta"] for t in two]), one["theta"], rtol=1e-4, atol=1e-5)
    key = "mean" if case == "es" else "eta"
    for t in two:
        np.testing.assert_allclose(t[key], one[key], rtol=0, atol=1e-6)
    if "buf_active" in one:
        for t in two:
            assert np.array_equal(t["buf_active"], one["buf_active"])
            assert np.array_equal(t["buf_new"], one["buf_new"])
            np.testing.assert_allclose(t["buf_score"], one["buf_score"], rtol=0, atol=1e-6)
