#!/bin/bash
# Round 5: the weight-gradient scatter (toued_gather_add) and the embedding partials' sum (toued_sum_rows_add) as one
# launch each: the meta-gradient tests, then C2
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t43 \
  "par:600:python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_curve.py tests/test_gpu_fullsize.py tests/test_gpu_debug.py tests/test_gpu_c5.py -q -x --timeout 300 --timeout-method thread" \
  "c2:300:$C && $C && $C"
