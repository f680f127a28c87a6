#!/bin/bash
# Round 6, call 2: the saves as 16-byte stores / loads in a unit-quad layout (FWD_QST, timing: the reduction still reads
# slab blocks) against the default, forward and backward at the C2 shape
B="python tools/bench_gru.py --which both"
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r06t2 \
  "ab:300:for i in 1 2 3; do $B; TOUED_LIB=${E}FWD_QST_1.so $B; done"
