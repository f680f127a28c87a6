#!/bin/bash
# Round 5: A/B of the spread DG stores (default) against the burst stores, stamps of both
B="python tools/bench_gru.py --which bwd"
E=to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r05t3 \
  "ab:300:$B && TOUED_LIB=${E}BWD_SPREAD_0.so $B && $B && TOUED_LIB=${E}BWD_SPREAD_0.so $B" \
  "stamps:120:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py && TOUED_LIB=${E}BWD_SPREAD_0_BWD_STAMPS_1.so python tools/bwd_stamps.py"
