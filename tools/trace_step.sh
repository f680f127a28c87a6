#!/bin/bash
# Kernel trace of a short bench run (for the per-step timeline: tools/step_timeline.py)
#   gpurun -- bash tools/trace_step.sh <tag>
set -euo pipefail
TAG=${1:-dev}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/trace_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- python3 "$R/bench.py" --steps ${STEPS:-3} \
    --warmup 2 --no_cpu_baseline --workloads none > "$OUT/bench.log" 2>&1
python3 "$R/tools/step_timeline.py" "$OUT" > "$OUT/timeline.txt"
rm -f "$OUT"/*.db
find "$OUT" -name "*kernel_trace.csv" -exec gzip -f {} \;
cat "$OUT/timeline.txt"
