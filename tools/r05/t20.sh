#!/bin/bash
# Round 5: the backward as two CU-masked half-grid launches out of phase (TOUED_BWD_HALVES=q)
B="python tools/bench_gru.py --which bwd"
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t20 \
  "par:300:TOUED_BWD_HALVES=5 python -u -m pytest tests/test_gpu_meta.py -q -x --timeout 120 --timeout-method thread -k 'backward_fused or meta_step_matches'" \
  "ab:400:for i in 1 2; do $B; TOUED_BWD_HALVES=0 $B; TOUED_BWD_HALVES=3 $B; TOUED_BWD_HALVES=5 $B; TOUED_BWD_HALVES=7 $B; done" \
  "c2:300:$C; TOUED_BWD_HALVES=5 $C"
