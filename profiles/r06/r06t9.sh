#!/bin/bash
# Round 6, call 9: phase stamps of the backward and forward on the unit-quad saves; a C2 step kernel trace
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r06t9 \
  "bst:200:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "fst:200:TOUED_LIB=${E}FWD_STAMPS_1.so python tools/fwd_stamps.py && TOUED_LIB=${E}FWD_STAMPS_1.so python tools/fwd_stamps.py --multi" \
  "trace:400:bash tools/trace_step.sh r06t9"
