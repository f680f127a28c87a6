#!/bin/bash
# Round 5: eval_agent's key chain started right after the last LPG forward (TOUED_EVAL_PREP=forwards, default) against
# at the reverse loop: parity, C2 A/B, a trace of the new order
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t50 \
  "par:600:python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_curve.py tests/test_gpu_fullsize.py -q -x --timeout 300 --timeout-method thread" \
  "c2:600:TOUED_EVAL_PREP=reverse $C && $C && TOUED_EVAL_PREP=reverse $C && $C && TOUED_EVAL_PREP=reverse $C && $C" \
  "trace:400:bash tools/trace_step.sh r05e"
