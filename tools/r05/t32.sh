#!/bin/bash
# Round 5: the next gate's first piece written during a pass's last k-steps (BWD_INPASS): parity, A/B, stamps, C2
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python tools/bench_gru.py --which bwd"
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t32 \
  "par:300:TOUED_LIB=${E}BWD_INPASS_1.so python -u -m pytest tests/test_gpu_meta.py -q -x --timeout 200 --timeout-method thread -k 'backward or meta_step_matches'" \
  "ab:300:for i in 1 2 3; do $B; TOUED_LIB=${E}BWD_INPASS_1.so $B; done" \
  "st:200:TOUED_LIB=${E}BWD_INPASS_1_BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "c2:300:$C && TOUED_LIB=${E}BWD_INPASS_1.so $C"
