#!/bin/bash
# Kernel trace of C3 regret rounds (tools/regret_round.py) and the last round's timeline (tools/round_timeline.py)
#   gpurun -- bash tools/trace_round.sh <tag>
set -euo pipefail
TAG=${1:-dev}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/round_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- python3 "$R/tools/regret_round.py" 3 \
    > "$OUT/round.log" 2>&1
python3 "$R/tools/round_timeline.py" "$OUT" > "$OUT/timeline.txt"
rm -f "$OUT"/*.db
find "$OUT" -name "*kernel_trace.csv" -exec gzip -f {} \;
cat "$OUT/round.log" | tail -4
cat "$OUT/timeline.txt"
