#!/bin/bash
# SQ counter passes (MFMA busy, issue mix, LDS conflicts) over the GRU, weight-gradient and rollout micro-benchmarks:
#   gpurun -- bash tools/pmc_kernels.sh r02
# Each pass is its own rocprofv3 run (at most 8 SQ counters + GRBM per pass, MI355X_MICROARCH.md); the
# summary (per kernel: mean counter value per launch) goes to gpurun_out/pmc_<tag>/summary.txt.
set -euo pipefail
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
B="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
i=0
for prog in "tools/bench_gru.py --which both --iters 1" "tools/bench_wgrad.py 3276800" "tools/bench_rollout.py --iters 1"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $A --kernel-trace -d "$OUT/a$i" -o run -- python3 $R/$prog > "$OUT/a$i.log" 2>&1
  echo "pass a$i done"
  timeout -s KILL 120 rocprofv3 --pmc $B --kernel-trace -d "$OUT/b$i" -o run -- python3 $R/$prog > "$OUT/b$i.log" 2>&1
  echo "pass b$i done"
done
python3 - "$OUT" > "$OUT/summary.txt" <<'PY'
import collections, glob, sqlite3, sys
out = sys.argv[1]
agg = collections.defaultdict(list)
for db in sorted(glob.glob(f"{out}/*/*.db")):
    c = sqlite3.connect(db)
    try:
        rows = c.execute("select kernel_name, counter_name, value from counters_collection").fetchall()
    except sqlite3.Error:
        continue
    for k, n, v in rows:
        k = k.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        if any(s in k for s in ("gru", "wgrad", "rollout")):
            agg[(k, n)].append(v)
for (k, n), v in sorted(agg.items()):
    print(f"{k:34s} {n:28s} {sum(v)/len(v):.6g}  (n={len(v)})")
PY
cat "$OUT/summary.txt"
find "$OUT" -name "*.db" -delete
