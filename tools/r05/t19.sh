#!/bin/bash
# Round 5: the backward's DG store placement (BWD_SPLACE): parity, A/B, stamps, the C2 step
B="python tools/bench_gru.py --which bwd"
E=$(pwd)/to-ued_amd/exp/libtoued_
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t19 \
  "par:300:TOUED_LIB=${E}BWD_SPLACE_1.so python -u -m pytest tests/test_gpu_meta.py -q -x --timeout 120 --timeout-method thread -k 'backward or meta_step_matches'" \
  "ab:300:for i in 1 2 3; do $B; TOUED_LIB=${E}BWD_SPLACE_1.so $B; done" \
  "st:200:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py && TOUED_LIB=${E}BWD_SPLACE_1_BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "c2:300:for i in 1 2; do $C; TOUED_LIB=${E}BWD_SPLACE_1.so $C; done"
