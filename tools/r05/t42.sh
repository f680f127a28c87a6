#!/bin/bash
# Round 5: toued_agent_step_entropy copies theta_k -> theta_{k+1} in its own blocks (no side-stream copies, no
# cross-stream waits in the update loop): parity, C2 A/B against the launch + side-copy path
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t42 \
  "par:600:python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_curve.py tests/test_gpu_es.py tests/test_gpu_debug.py -q -x --timeout 300 --timeout-method thread" \
  "c2:500:TOUED_STEP_ENTROPY=0 $C && $C && TOUED_STEP_ENTROPY=0 $C && $C && TOUED_STEP_ENTROPY=0 $C && $C"
