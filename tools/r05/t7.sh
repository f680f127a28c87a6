#!/bin/bash
# Round 5: what the refill windows between the backward's gate passes wait on (timing-only variants)
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r05t7 \
  "st0:120:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "st1:120:TOUED_LIB=${E}BWD_STAMPS_1_BWD_TREFILL_1.so python tools/bwd_stamps.py" \
  "st2:120:TOUED_LIB=${E}BWD_STAMPS_1_BWD_TREFILL_2.so python tools/bwd_stamps.py"
