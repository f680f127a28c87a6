#!/bin/bash
# Round 5: C4 forward with the ring / x declared back in the step loop; order and head-deferral variants; C2 forward
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python tools/bench_fwd_multi.py"
F="python tools/bench_gru.py --which fwd"
bash tools/gpu_steps.sh r05t34 \
  "ab:400:for i in 1 2; do $B; TOUED_LIB=${E}FWD_XFIRST_1.so $B; TOUED_LIB=${E}FWD_HDEFER_0.so $B; done" \
  "c2f:200:for i in 1 2; do $F; TOUED_LIB=${E}FWD_HDEFER_0.so $F; done"
