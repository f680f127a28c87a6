#!/bin/bash
# Round 5: k_rows_sorted's phase-1 warm-up (the samples' index words and table rows in flight together, ROWS_WARM):
# parity, C2 A/B against a ROWS_WARM=0 build
E=$(pwd)/to-ued_amd/exp/libtoued_
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t48 \
  "par:600:python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_es.py -q -x --timeout 300 --timeout-method thread" \
  "c2:600:TOUED_LIB=${E}ROWS_WARM_0.so $C && $C && TOUED_LIB=${E}ROWS_WARM_0.so $C && $C && TOUED_LIB=${E}ROWS_WARM_0.so $C && $C"
