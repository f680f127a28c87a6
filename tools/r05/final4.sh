#!/bin/bash
# Round 5 (final, step-level fusions + one-launch scatter and partial sums): smoke, the default bench (all workloads, CPU baselines), then the profiles
# (kernel stats, FETCH/WRITE PMC passes) -- the -m gpu suite ran on this tree in r05t46 (195 passed)
bash tools/gpu_steps.sh r05final4 \
  "smoke:150:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py" \
  "prof:1000:bash tools/profile.sh r05"
