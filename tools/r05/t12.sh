#!/bin/bash
# Round 5: the backward's next-step prefetch (BWD_PF leading quads, BWD_PFX tile 0's x, issued in the dhn pass)
B="python tools/bench_gru.py --which bwd"
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r05t12 \
  "ab:400:for i in 1 2; do $B; TOUED_LIB=${E}BWD_PF_1.so $B; TOUED_LIB=${E}BWD_PF_2.so $B; TOUED_LIB=${E}BWD_PF_2_BWD_PFX_1.so $B; TOUED_LIB=${E}BWD_PF_1_BWD_PFX_1.so $B; done" \
  "par:300:TOUED_LIB=${E}BWD_PF_2_BWD_PFX_1.so python -u -m pytest tests/test_gpu_meta.py -q -x --timeout 120 --timeout-method thread -k 'backward or meta_step_matches'"
