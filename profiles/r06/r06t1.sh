#!/bin/bash
# Round 6, call 1: the new production-size C4 tests and the fallback-equivalence test; the recompute-backward timing
# prototype (BWD_TRECOMP) against the default, with stamps; C4's fragment-stream ceiling (FWD_CAND0)
B="python tools/bench_gru.py --which bwd"
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r06t1 \
  "tests:700:python -u -m pytest tests/test_gpu_es_fullsize.py tests/test_gpu_fallbacks.py -x -v --timeout 400 --timeout-method thread" \
  "bwd:300:for i in 1 2; do $B; TOUED_LIB=${E}BWD_TRECOMP_1.so $B; done" \
  "st:200:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py && TOUED_LIB=${E}BWD_STAMPS_1_BWD_TRECOMP_1.so python tools/bwd_stamps.py" \
  "c4k:200:for i in 1 2; do python tools/bench_fwd_multi.py; TOUED_LIB=${E}FWD_CAND0_1.so python tools/bench_fwd_multi.py; done" \
  "c4s:400:python tools/es_step.py 2 && TOUED_LIB=${E}FWD_CAND0_1.so python tools/es_step.py 2"
