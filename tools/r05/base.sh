#!/bin/bash
# Round 5 baseline on a fresh box: the C2 headline alone (no CPU baseline, no C3/C4)
bash tools/gpu_steps.sh r05base \
  "bench:300:python bench.py --no_cpu_baseline --workloads none --steps 10"
