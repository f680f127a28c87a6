#!/bin/bash
# Round 4 (x): the backward's head-cotangent loads of step t+1 issued in step t's tail (BWD_HEAD_AHEAD=1, the
# default build) against BWD_HEAD_AHEAD=0: micro timings, stamps, parity, C2
E=to-ued_amd/exp/libtoued_
B="python tools/bench_gru.py --which bwd"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_steps.sh r04x \
  "v1:120:$B && $B" \
  "v0:120:TOUED_LIB=${E}BWD_HEAD_AHEAD_0.so $B && TOUED_LIB=${E}BWD_HEAD_AHEAD_0.so $B" \
  "v1b:120:$B" \
  "s1:120:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "s0:120:TOUED_LIB=${E}BWD_STAMPS_1_BWD_HEAD_AHEAD_0.so python tools/bwd_stamps.py" \
  "par:400:$T tests/test_gpu_meta.py" \
  "c1:200:python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "c0:200:TOUED_LIB=${E}BWD_HEAD_AHEAD_0.so python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "c1b:200:python bench.py --no_cpu_baseline --workloads none --steps 10"
