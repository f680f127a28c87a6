#!/bin/bash
# Round 5: the C4 per-candidate forward regression (2.22 -> 2.65 ms): head deferral / lead-load order variants
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python tools/bench_fwd_multi.py"
bash tools/gpu_steps.sh r05t33 \
  "ab:400:for i in 1 2; do $B; TOUED_LIB=${E}FWD_HDEFER_0.so $B; TOUED_LIB=${E}FWD_XFIRST_1.so $B; TOUED_LIB=${E}FWD_HDEFER_0_FWD_XFIRST_1.so $B; done"
