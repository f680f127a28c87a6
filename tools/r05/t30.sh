#!/bin/bash
# Round 5: phase stamps of the backward and the forward on the slab-layout tree
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r05t30 \
  "bst:200:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "fst:200:TOUED_LIB=${E}FWD_STAMPS_1.so python tools/fwd_stamps.py"
