#!/bin/bash
# Round 5: rollout 0's draws first, the other batches' on the side stream beside it (TOUED_DRAWS_AHEAD): parity, C2 A/B
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t47 \
  "par:600:python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_curve.py tests/test_gpu_env.py tests/test_gpu_c5.py -q -x --timeout 300 --timeout-method thread" \
  "c2:600:TOUED_DRAWS_AHEAD=0 $C && $C && TOUED_DRAWS_AHEAD=0 $C && $C && TOUED_DRAWS_AHEAD=0 $C && $C"
