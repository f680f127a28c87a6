#!/bin/bash
# Round 5: spread DG stores in the backward passes (BWD_SPREAD=1 default) against the burst stores (BWD_SPREAD=0):
# parity, A/B timings, per-phase and per-wave stamps, then the C2 bench
B="python tools/bench_gru.py --which bwd"
E=to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r05t2 \
  "dbg:300:python -u -m pytest tests/test_gpu_debug.py -v -x --timeout 200 --timeout-method thread" \
  "par:400:python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_fullsize.py -x -q -s --timeout 200 --timeout-method thread" \
  "ab:300:$B && TOUED_LIB=${E}BWD_SPREAD_0.so $B && $B && TOUED_LIB=${E}BWD_SPREAD_0.so $B" \
  "stamps:120:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py && TOUED_LIB=${E}BWD_SPREAD_0_BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "bench:300:python bench.py --no_cpu_baseline --workloads none --steps 10"
