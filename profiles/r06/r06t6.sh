#!/bin/bash
# Round 6, call 6: h_in back in slab blocks, r / z / hn in unit-quad blocks; which 16-byte store form is deterministic;
# kernel timings against the previous commit
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python tools/bench_gru.py --which both"
bash tools/gpu_steps.sh r06t6 \
  "b128nt:120:python tools/det_fwd_diff.py" \
  "b64:120:TOUED_LIB=${E}GRU_ST4_MODE_1.so python tools/det_fwd_diff.py" \
  "b32:120:TOUED_LIB=${E}GRU_ST4_MODE_2.so python tools/det_fwd_diff.py" \
  "b128:120:TOUED_LIB=${E}GRU_ST4_MODE_3.so python tools/det_fwd_diff.py" \
  "ab:300:for i in 1 2; do $B; TOUED_LIB=${E}GRU_ST4_MODE_1.so $B; TOUED_LIB=${E}head.so $B; done"
