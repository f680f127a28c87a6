#!/bin/bash
# Round 5: the parameter-history ring (no theta_K copy back), one-block-per-table masked inits; the full -m gpu suite,
# then C2 with the reverse pair on and off
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t38 \
  "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "c2:500:TOUED_REVERSE_PAIR=0 $C && $C && TOUED_REVERSE_PAIR=0 $C && $C && TOUED_REVERSE_PAIR=0 $C && $C"
