#!/bin/bash
# Round 5: the backward's A-fragment ring depth (BWD_RD 4 / 6 / 8) with and without the spread DG stores
B="python tools/bench_gru.py --which bwd"
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r05t8 \
  "ab:400:for i in 1 2; do $B; TOUED_LIB=${E}BWD_SPREAD_0.so $B; TOUED_LIB=${E}BWD_SPREAD_0_BWD_RD_8.so $B; TOUED_LIB=${E}BWD_RD_8.so $B; TOUED_LIB=${E}BWD_SPREAD_0_BWD_RD_6.so $B; done" \
  "st:120:TOUED_LIB=${E}BWD_SPREAD_0_BWD_RD_8_BWD_STAMPS_1.so python tools/bwd_stamps.py && TOUED_LIB=${E}BWD_RD_8_BWD_STAMPS_1.so python tools/bwd_stamps.py"
B="python tools/bench_gru.py --which bwd"
F="python tools/bench_gru.py --which fwd"
bash tools/gpu_steps.sh r05t8b \
  "tnotr:200:$B && TOUED_LIB=${E}BWD_TNOTR_1.so $B && TOUED_LIB=${E}BWD_TNOTR_1_BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "fwd16:200:$F && TOUED_LIB=${E}FWD_TST16_1.so $F && $F && TOUED_LIB=${E}FWD_TST16_1.so $F"
