#!/bin/bash
# Round 6, call 10: gru.hip with SLP vectorisation on (packed FP32), the forward without saves (FWD_NOSAVE=1), against
# the default build
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python tools/bench_gru.py --which both"
bash tools/gpu_steps.sh r06t10 \
  "ab:300:for i in 1 2; do $B; TOUED_LIB=${E}slp.so $B; TOUED_LIB=${E}FWD_NOSAVE_1.so $B; done"
