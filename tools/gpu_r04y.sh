#!/bin/bash
# Round 4 (y): the forward's done flags loaded with x(t) before the contraction (FWD_DONE_EARLY=1, the default build)
# against FWD_DONE_EARLY=0: micro timings, stamps, parity (meta + ES), C2 and C4
E=to-ued_amd/exp/libtoued_
B="python tools/bench_gru.py --which fwd"
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh r04y \
  "v1:120:$B && $B" \
  "v0:120:TOUED_LIB=${E}FWD_DONE_EARLY_0.so $B && TOUED_LIB=${E}FWD_DONE_EARLY_0.so $B" \
  "s1:120:TOUED_LIB=${E}FWD_STAMPS_1.so python tools/fwd_stamps.py" \
  "s0:120:TOUED_LIB=${E}FWD_STAMPS_1_FWD_DONE_EARLY_0.so python tools/fwd_stamps.py" \
  "par:600:$T tests/test_gpu_meta.py tests/test_gpu_es.py" \
  "c1:200:python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "c0:200:TOUED_LIB=${E}FWD_DONE_EARLY_0.so python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "c1b:200:python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "c0b:200:TOUED_LIB=${E}FWD_DONE_EARLY_0.so python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "es1:300:python bench.py --no_cpu_baseline --workloads c4 --steps 2" \
  "es0:300:TOUED_LIB=${E}FWD_DONE_EARLY_0.so python bench.py --no_cpu_baseline --workloads c4 --steps 2"
