"""Summarise the rocprofv3 databases written by tools/profile.sh into profiles/<tag>/.

    python tools/prof_summary.py gpurun_out/prof_r01 profiles/r01

Writes:
  kernel_stats.csv   per kernel: calls, total/avg/min/max duration (ns), share of GPU time
                     (kernel-trace pass, bench.py --steps 3 --warmup 2 incl. warmup)
  pmc_traffic.json   per kernel: mean FETCH_SIZE / WRITE_SIZE per launch (raw, kB) and the
                     corrected HBM bytes per launch using the factors measured by the calibration
                     kernels (tools/calib_fetch.hip streams exactly 1 GiB per launch)
"""
from __future__ import annotations

import csv
import json
import sqlite3
import sys
from collections import defaultdict
from pathlib import Path

GIB = float(1 << 30)


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0]


def kernel_stats(db: Path):
    c = sqlite3.connect(db)
    agg = defaultdict(list)
    for name, dur in c.execute("select name, duration from kernels"):
        agg[short(name)].append(float(dur))
    tot = sum(sum(v) for v in agg.values())
    rows = []
    for k, v in agg.items():
        # median beside the mean: the bench's first (warmup) launches under the profiler run cold and slow
        srt = sorted(v)
        med = srt[len(srt) // 2] if len(srt) % 2 else 0.5 * (srt[len(srt) // 2 - 1] + srt[len(srt) // 2])
        rows.append({"kernel": k, "calls": len(v), "total_ns": round(sum(v)), "avg_ns": round(sum(v) / len(v), 1),
                     "median_ns": round(med, 1), "min_ns": round(min(v)), "max_ns": round(max(v)),
                     "percent": round(100 * sum(v) / tot, 3)})
    rows.sort(key=lambda r: -r["total_ns"])
    return rows


def pmc(db: Path, counter: str):
    c = sqlite3.connect(db)
    agg = defaultdict(list)
    for name, val in c.execute("select kernel_name, value from counters_collection where counter_name = ?",
                               (counter,)):
        agg[short(name)].append(float(val))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    dst.mkdir(parents=True, exist_ok=True)
    rows = kernel_stats(src / "ks" / "run_results.db")
    with open(dst / "kernel_stats.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    if (src / "ks_wl" / "run_results.db").exists():      # the C3 / C4 workloads' kernel trace (bench.py --workloads)
        wl = kernel_stats(src / "ks_wl" / "run_results.db")
        with open(dst / "kernel_stats_workloads.csv", "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(wl[0]))
            w.writeheader()
            w.writerows(wl)
    cf = pmc(src / "calib_fetch" / "run_results.db", "FETCH_SIZE")
    cw = pmc(src / "calib_write" / "run_results.db", "WRITE_SIZE")
    # factor = true bytes / (counter kB * 1024)
    f_b32 = GIB / (cf["rd_b32"] * 1024.0)
    f_b128 = GIB / (cf["rd_b128"] * 1024.0)
    w_b32 = GIB / (cw["wr_b32"] * 1024.0)
    fetch = pmc(src / "pmc_fetch" / "run_results.db", "FETCH_SIZE")
    write = pmc(src / "pmc_write" / "run_results.db", "WRITE_SIZE")
    out = {"calibration": {"fetch_factor_b32": round(f_b32, 4), "fetch_factor_b128": round(f_b128, 4),
                           "write_factor_b32": round(w_b32, 4),
                           "note": "true bytes = counter kB * 1024 * factor; measured on 1 GiB streams"},
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        fb = fetch.get(k, 0.0) * 1024.0
        wb = write.get(k, 0.0) * 1024.0
        out["kernels"][k] = {"fetch_kB_raw": round(fetch.get(k, 0.0), 1), "write_kB_raw": round(write.get(k, 0.0), 1),
                             "hbm_bytes_per_launch": round(fb * f_b32 + wb * w_b32)}
    (dst / "pmc_traffic.json").write_text(json.dumps(out, indent=1))
    for r in rows[:12]:
        print(r)
    print(json.dumps(out["calibration"]))
    for k in ("k_gru_bwd6n<true>", "k_gru_fwd6<true>", "k_wgrad_h3<8, 2, 3>"):
        print(k, out["kernels"].get(k))


if __name__ == "__main__":
    main()
