#!/bin/bash
# SQ counter passes over the GRU micro-benchmark (tools/bench_gru.py):  gpurun -- bash tools/pmc_gru.sh bwd
set -euo pipefail
WHICH=${1:-bwd}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_gru_$WHICH
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 python3 "$R/tools/bench_gru.py" --which "$WHICH" --iters 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS --kernel-trace -d "$OUT/a" -o run -- \
    python3 "$R/tools/bench_gru.py" --which "$WHICH" --iters 1 > "$OUT/a.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD \
    SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace \
    -d "$OUT/b" -o run -- python3 "$R/tools/bench_gru.py" --which "$WHICH" --iters 1 > "$OUT/b.log" 2>&1
python3 - "$OUT" <<'PY'
import sqlite3, sys, glob, collections
out = sys.argv[1]
for sub in ("a", "b"):
    for db in glob.glob(f"{out}/{sub}/*.db"):
        c = sqlite3.connect(db)
        agg = collections.defaultdict(list)
        for k, n, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
            if "gru" in k:
                agg[(k.split("(")[0].replace("(anonymous namespace)::", ""), n)].append(v)
        for (k, n), v in sorted(agg.items()):
            print(f"{k:40s} {n:28s} {sum(v)/len(v):.4g}")
PY
