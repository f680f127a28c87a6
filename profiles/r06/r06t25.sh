#!/bin/bash
# Round 6, call 25: where the ping-pong forward's step goes -- per-half work and barrier waits (FWD_PP stamps) beside
# the lockstep forward's phase stamps on the same box
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r06t25 \
  "pp:200:TOUED_LIB=${E}FWD_PP_1_FWD_STAMPS_1.so python tools/fwd_stamps.py --pp" \
  "ls:200:TOUED_LIB=${E}FWD_STAMPS_1.so python tools/fwd_stamps.py"
