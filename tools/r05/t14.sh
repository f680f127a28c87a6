#!/bin/bash
# Round 5: the backward's first-round stagger (TOUED_BWD_STAGGER quanta,mode) and the forward's lead-load order
B="python tools/bench_gru.py --which bwd"
F="python tools/bench_gru.py --which fwd"
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r05t14 \
  "ab:500:for i in 1 2; do $B; TOUED_BWD_STAGGER=5,0 $B; TOUED_BWD_STAGGER=5,1 $B; TOUED_BWD_STAGGER=2,2 $B; TOUED_BWD_STAGGER=3,0 $B; TOUED_BWD_STAGGER=8,0 $B; done" \
  "fwd:200:for i in 1 2 3; do $F; TOUED_LIB=${E}FWD_XFIRST_1.so $F; done" \
  "st:200:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py && TOUED_BWD_STAGGER=5,0 TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py"
