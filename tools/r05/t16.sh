#!/bin/bash
# Round 5: k_wgrad_h3 with B's raw slabs through a two-buffer register ring (H3_BR2): parity, alone, in the C2 step
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t16 \
  "par:300:TOUED_LIB=${E}H3_BR2_1.so python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_fullsize.py -q -x --timeout 200 --timeout-method thread" \
  "wg:300:for i in 1 2; do python tools/bench_wgrad.py; TOUED_LIB=${E}H3_BR2_1.so python tools/bench_wgrad.py; done" \
  "c2:400:for i in 1 2; do $B; TOUED_LIB=${E}H3_BR2_1.so $B; done"
