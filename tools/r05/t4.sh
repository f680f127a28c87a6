#!/bin/bash
# Round 5: per-wave pass stamps of the backward (spread and burst DG stores)
E=to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r05t4 \
  "stamps:120:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py && TOUED_LIB=${E}BWD_SPREAD_0_BWD_STAMPS_1.so python tools/bwd_stamps.py"
