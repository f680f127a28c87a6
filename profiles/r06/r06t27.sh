#!/bin/bash
# Round 6, call 27: inside the lockstep forward's gate maths (sub-stamps: done flags + gate_ain, each row tile, the
# head fold), with the done flags loaded at the step start (FWD_DNF_EARLY) against the default; forward timing A/B
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python tools/bench_gru.py --which fwd"
bash tools/gpu_steps.sh r06t27 \
  "st:200:TOUED_LIB=${E}FWD_STAMPS_1.so python tools/fwd_stamps.py --gm && TOUED_LIB=${E}FWD_STAMPS_1_FWD_DNF_EARLY_1.so python tools/fwd_stamps.py --gm" \
  "ab:300:for i in 1 2 3; do $B; TOUED_LIB=${E}FWD_DNF_EARLY_1.so $B; done"
