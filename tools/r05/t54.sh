#!/bin/bash
# Round 5: k_sum_rows_add as one workgroup per column with a fixed-order tree (it was one serial thread per column:
# 0.18 ms): parity, C2, a trace
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t54 \
  "par:600:python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_curve.py -q -x --timeout 300 --timeout-method thread" \
  "c2:300:$C && $C" \
  "trace:400:bash tools/trace_step.sh r05f"
