#!/bin/bash
# One GPU-box pass used during development: the -m gpu suite, then the micro-benchmarks and the headline bench.
#   gpurun -- bash tools/gpu_round.sh <tag> [pytest -k expression]
# Every step has its own time limit and the chain stops at the first failure.
set -euo pipefail
TAG=${1:-dev}
K=${2:-}
O=gpurun_out/$TAG
mkdir -p "$O"
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > "$O/gputest.log" 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gputest.log" 2>&1
fi
tail -2 "$O/gputest.log"
timeout -k 10 120 python tools/bench_rollout.py --iters 3 > "$O/rollout.json" 2>&1; tail -1 "$O/rollout.json"
timeout -k 10 120 python tools/bench_wgrad.py > "$O/wgrad.json" 2>&1; tail -1 "$O/wgrad.json"
timeout -k 10 120 python tools/bench_gru.py --which both > "$O/gru.json" 2>&1; tail -1 "$O/gru.json"
timeout -k 10 300 python bench.py --no_cpu_baseline > "$O/bench.json" 2>&1; tail -1 "$O/bench.json"
