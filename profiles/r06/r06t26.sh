#!/bin/bash
# Round 6, call 26: the ping-pong forward with the gate maths at issue priority 2 over the partner's contraction:
# stamps and forward timing against the default
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python tools/bench_gru.py --which fwd"
bash tools/gpu_steps.sh r06t26 \
  "pp:200:TOUED_LIB=${E}FWD_PP_1_FWD_STAMPS_1_FWD_PP_PRIO_2.so python tools/fwd_stamps.py --pp" \
  "ab:300:for i in 1 2; do $B; TOUED_LIB=${E}FWD_PP_1_FWD_PP_PRIO_2.so $B; done"
