#!/bin/bash
# Round 4 (n): the backward's early ring fill (BWD_PRE=1) against the default: micro timings, stamps, parity, C2
E=to-ued_amd/exp/libtoued_
B="python tools/bench_gru.py --which bwd"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_steps.sh r04n \
  "v0:120:$B && $B" \
  "v1:120:TOUED_LIB=${E}BWD_PRE_1.so $B && TOUED_LIB=${E}BWD_PRE_1.so $B" \
  "v0b:120:$B" \
  "s0:120:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "s1:120:TOUED_LIB=${E}BWD_STAMPS_1_BWD_PRE_1.so python tools/bwd_stamps.py" \
  "par:400:TOUED_LIB=${E}BWD_PRE_1.so $T tests/test_gpu_meta.py" \
  "c1:200:TOUED_LIB=${E}BWD_PRE_1.so python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "c0:200:python bench.py --no_cpu_baseline --workloads none --steps 10"
