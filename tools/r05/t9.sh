#!/bin/bash
# Round 5: issue priority of the two waves per SIMD in the backward's memory part
B="python tools/bench_gru.py --which bwd"
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r05t9 \
  "ab:300:for i in 1 2; do $B; TOUED_LIB=${E}BWD_MPRIO_1.so $B; TOUED_LIB=${E}BWD_MPRIO_2.so $B; done" \
  "st:200:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py && TOUED_LIB=${E}BWD_MPRIO_1_BWD_STAMPS_1.so python tools/bwd_stamps.py && TOUED_LIB=${E}BWD_MPRIO_2_BWD_STAMPS_1.so python tools/bwd_stamps.py"
