#!/bin/bash
# Round 6, call 24: the ping-pong forward (FWD_PP=1: the workgroup's two halves one interval apart, each SIMD's gate
# maths beside its partner's matrix work): forward timing against the default, the GRU parity tests on the variant,
# the C2 bench
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python tools/bench_gru.py --which fwd"
C="python bench.py --workloads none --no_cpu_baseline --steps 10"
bash tools/gpu_steps.sh r06t24 \
  "ab:300:for i in 1 2; do $B; TOUED_LIB=${E}FWD_PP_1.so $B; done" \
  "par:600:TOUED_LIB=${E}FWD_PP_1.so python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread" \
  "c2:400:$C && TOUED_LIB=${E}FWD_PP_1.so $C && $C && TOUED_LIB=${E}FWD_PP_1.so $C"
