#!/bin/bash
# Focused PMC passes over the GRU kernels (tools/bench_gru.py): issue/stall breakdown and TA pressure.
#   gpurun -- bash tools/pmc_bwd.sh [which=bwd]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
W=${1:-bwd}
OUT=$R/gpurun_out/pmc_$W
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM TA_BUSY_avr TA_BUSY_max"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_gru_${W}6" --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/tools/bench_gru.py" --which $W --iters 1 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
