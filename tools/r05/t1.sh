#!/bin/bash
# Round 5: the new GPU tests (debug hooks, device error word, full-size float64 checks), then the whole suite and the bench
bash tools/gpu_steps.sh r05t1 \
  "new:400:python -u -m pytest tests/test_gpu_debug.py tests/test_gpu_fullsize.py -v -x --timeout 300 --timeout-method thread" \
  "suite:700:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "bench:300:python bench.py --no_cpu_baseline --workloads none --steps 10"
