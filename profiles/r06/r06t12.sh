#!/bin/bash
# Round 6, call 12: packed FP32 (v_pk_*_f32) in the backward's memory part (BWD_PK) and the forward's head partials
# (FWD_PK): kernel timings against the default, C4's per-candidate forward, and the GRU parity tests on the variant
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python tools/bench_gru.py --which both"
bash tools/gpu_steps.sh r06t12 \
  "ab:300:for i in 1 2; do $B; TOUED_LIB=${E}BWD_PK_1.so $B; TOUED_LIB=${E}BWD_PK_1_FWD_PK_1.so $B; done" \
  "c4k:200:for i in 1 2; do python tools/bench_fwd_multi.py; TOUED_LIB=${E}BWD_PK_1_FWD_PK_1.so python tools/bench_fwd_multi.py; done" \
  "par:600:TOUED_LIB=${E}BWD_PK_1_FWD_PK_1.so python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_fullsize.py tests/test_gpu_es.py -x -q --timeout 300 --timeout-method thread"
