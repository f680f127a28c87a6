#!/bin/bash
# Round 6, call 7: b128 saves with s_nop wait states after each store (GRU_ST4_MODE 4: s_nop 1, 5: s_nop 4) --
# determinism (three forwards) and kernel timings against b64 stores and the previous commit
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python tools/bench_gru.py --which both"
bash tools/gpu_steps.sh r06t7 \
  "nop1:120:for i in 1 2 3; do TOUED_LIB=${E}GRU_ST4_MODE_4.so python tools/det_fwd_diff.py; done" \
  "nop4:120:for i in 1 2 3; do TOUED_LIB=${E}GRU_ST4_MODE_5.so python tools/det_fwd_diff.py; done" \
  "ab:300:for i in 1 2; do TOUED_LIB=${E}GRU_ST4_MODE_4.so $B; TOUED_LIB=${E}GRU_ST4_MODE_5.so $B; TOUED_LIB=${E}GRU_ST4_MODE_1.so $B; TOUED_LIB=${E}head.so $B; done"
