"""Per-phase timing of the per-agent sorted-row kernels from in-kernel s_memtime stamps (a ROWS_STAMPS=1 variant):

    python tools/build_variant.py agent.hip ROWS_STAMPS=1
    TOUED_LIB=to-ued_amd/exp/libtoued_ROWS_STAMPS_1.so python tools/rows_stamps.py

Runs two C2 meta-steps (512 agents, tabular, K = 5) and prints, for the first 64 blocks of each of the last step's
launches, the mean shader cycles of each phase: per-sample rows + partial sums, sort, segmented scan, the row writes
(read-modify-write of the touched rows), norms / clip / apply, entropy metrics.  Slot 0: the inner update
(k_rows_sorted<GradStepEntOp>); slots 1, 2: the reverse step's two bodies (k_rows_sorted2<EntropyClipOp, HvpOp>)."""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "to-ued_amd"))
import torch  # noqa: E402


def main():
    from toued import _lib
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = parse_args(["--env_mode", "tabular", "--num_agents", "512", "--num_mini_batches", "1"])
    tr = Trainer(args)
    for _ in range(2):
        tr.meta_step()
    torch.cuda.synchronize()
    fn = _lib.lib().toued_dbg_rows_stamps
    fn.argtypes = [ctypes.c_void_p]
    buf = np.zeros(3 * 8 * 64 * 8, np.uint64)
    assert fn(buf.ctypes.data) == 0
    st = buf.reshape(3, 8, 64, 8).astype(np.int64)
    names = ["rows + partials", "sort", "segmented scan", "row writes", "norms / clip / apply", "entropy metrics"]
    # per slot, the last step's launches (ring entries 5, 6, 7, 0, 1 of 10 launches per slot over the two steps; slot
    # 0 also holds k_rows_sorted<LpgLossOp>, the step's sixth one-op launch)
    for slot, kind in enumerate(["k_rows_sorted (GradStepEntOp; LpgLossOp)", "k_rows_sorted2 body 1 (EntropyClipOp)",
                                 "k_rows_sorted2 body 2 (HvpOp)"]):
        for ln in (5, 6, 7, 0, 1):
            e = st[slot, ln]
            if not e[:, 0].all():
                continue
            ph = np.diff(e, axis=1)[:, :6]
            res = {n: round(float(ph[:, i].mean())) for i, n in enumerate(names)}
            res["total"] = round(float((e[:, 6] - e[:, 0]).mean()))
            print(json.dumps({"kernel": kind, "launch": ln, **res}), flush=True)
    # every block's body start / end on the 100 MHz real-time clock and its placement, per launch: dispatch spread,
    # body durations, and how the late-starting blocks sit on the CUs (ring of 8 launches per slot; the last step's 5)
    sf = _lib.lib().toued_dbg_rows_span
    sf.argtypes = [ctypes.c_void_p]
    sp = np.zeros(3 * 8 * 1024 * 4, np.uint64)
    assert sf(sp.ctypes.data) == 0
    sp = sp.reshape(3, 8, 1024, 4).astype(np.int64)[:, :, :512]
    for slot in range(3):
        for ln in (5, 6, 7, 0, 1):
            e = sp[slot, ln]
            if not e[:, 0].all():
                continue
            s0 = e[:, 0].min()
            st_us, en_us = (e[:, 0] - s0) / 100.0, (e[:, 1] - s0) / 100.0
            cu = (e[:, 2] & 15) * 256 + ((e[:, 3] >> 8) & 255)   # XCC_ID, then SE / SH / CU of HW_ID
            late = st_us > 5.0
            per_cu = {c: int((cu == c).sum()) for c in np.unique(cu)}
            late_cus = np.unique(cu[late])
            print(json.dumps({
                "slot": slot, "launch": ln, "cus": len(per_cu),
                "blocks_per_cu": {str(k): v for k, v in sorted(
                    {n: sum(1 for x in per_cu.values() if x == n) for n in set(per_cu.values())}.items())},
                "late_blocks": int(late.sum()), "late_on_cus_with_early_blocks": int(sum(
                    1 for c in late_cus if (~late & (cu == c)).any())),
                "start_us_p50_p90_max": np.percentile(st_us, [50, 90, 100]).round(2).tolist(),
                "end_us_p50_p90_max": np.percentile(en_us, [50, 90, 100]).round(2).tolist(),
                "body_us_p50_p90_max": np.percentile(en_us - st_us, [50, 90, 100]).round(2).tolist(),
                "late_start_us": sorted(st_us[late].round(1).tolist())[:12],
                "abs_start_end_us": [round(float(s0) / 100.0, 2), round(float(e[:, 1].max()) / 100.0, 2)]}),
                flush=True)

if __name__ == "__main__":
    main()
