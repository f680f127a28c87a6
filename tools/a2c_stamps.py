"""Per-phase timing of k_a2c_update from in-kernel s_memtime stamps (an A2C_STAMPS=1 variant library):

    python tools/build_variant.py a2c.hip A2C_STAMPS=1
    TOUED_LIB=to-ued_amd/exp/libtoued_A2C_STAMPS_1.so python tools/a2c_stamps.py

Runs C3 regret rounds (512 antagonists, all_shortlife, W = 64, T = 20, 250 updates) and prints, over the last
launch's 512 workgroups, the mean shader-clock cycles of one update's phases: the env chain (k_a2c_chain; with
TOUED_A2C_CHAIN=0 the separate k_a2c_update's trajectory staging instead), GAE + normalisation, per-sample row
vectors + block sums, the 2048-key bitonic sort, the segmented sums, the two norms, clip + SGD."""
import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
import torch  # noqa: E402


def main():
    from toued import _lib
    from toued.env import L_LIFETIME
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = parse_args(["--env_mode", "all_shortlife", "--num_agents", "512", "--num_mini_batches", "1",
                       "--score_function", "alg_regret"])
    tr = Trainer(args)
    for _ in range(2):
        tr.agents.step = tr.agents.levels[:, L_LIFETIME].clone()
        tr.buffer, tr.agents = tr.sampler.sample(tr.rng, tr.buffer, tr.agents)
    torch.cuda.synchronize()
    buf = np.zeros(512 * 8, np.uint64)
    fn = _lib.lib().toued_dbg_a2c_stamps
    fn.argtypes = [ctypes.c_void_p]
    assert fn(buf.ctypes.data) == 0
    st = buf.reshape(512, 8).astype(np.int64)
    chain = os.environ.get("TOUED_A2C_CHAIN") != "0"
    res = {}
    if chain:   # k_a2c_chain's last update: slot 7 = end of the env phase
        res["env chain (T steps)"] = float((st[:, 7] - st[:, 0]).mean())
        res["V gather + GAE + normalise"] = float((st[:, 1] - st[:, 7]).mean())
    else:
        res["stage + GAE + normalise"] = float((st[:, 1] - st[:, 0]).mean())
    names = ["per-sample rows + block sums", "bitonic sort 2048", "segmented sums", "norms", "clip + SGD"]
    for i, n in enumerate(names):
        res[n] = float((st[:, i + 2] - st[:, i + 1]).mean())
    res["update total"] = float((st[:, 6] - st[:, 0]).mean())
    print(json.dumps({k: round(v) for k, v in res.items()}), flush=True)
    if hasattr(_lib.lib(), "toued_dbg_a2c_fine"):   # an A2C_STAMPS_FINE variant: inside the V gather + GAE phase
        fb = np.zeros(512 * 8, np.uint64)
        ff = _lib.lib().toued_dbg_a2c_fine
        ff.argtypes = [ctypes.c_void_p]
        assert ff(fb.ctypes.data) == 0
        f = fb.reshape(512, 8).astype(np.int64)
        names = ["barrier after the env chain", "V gather + barrier", "per-worker GAE scan", "mean / critic-loss sums",
                 "variance sum", "abar + barrier"]
        fine = {"env end -> F0": float((f[:, 0] - st[:, 7]).mean())}
        for i, n in enumerate(names[1:]):
            fine[n] = float((f[:, i + 1] - f[:, i]).mean())
        print(json.dumps({"fine": {k: round(v) for k, v in fine.items()}}), flush=True)


if __name__ == "__main__":
    main()
