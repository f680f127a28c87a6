#!/bin/bash
# Round 5 (final, step-level fusions): smoke, the default bench (all workloads, CPU baselines), then the profiles
# (kernel stats, FETCH/WRITE PMC passes) -- the -m gpu suite ran on this tree in r05t40 (193 passed)
bash tools/gpu_steps.sh r05final3 \
  "smoke:150:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py" \
  "prof:1000:bash tools/profile.sh r05"
