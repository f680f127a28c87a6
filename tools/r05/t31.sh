#!/bin/bash
# Round 5: the forward's deferred head reduce (FWD_HDEFER): parity, forward alone, the C2 step, C4, same box
E=$(pwd)/to-ued_amd/exp/libtoued_
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t31 \
  "par:400:python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_es.py tests/test_gpu_curve.py -q -x --timeout 200 --timeout-method thread" \
  "fwd:300:for i in 1 2; do python tools/bench_gru.py --which fwd; TOUED_LIB=${E}FWD_HDEFER_0.so python tools/bench_gru.py --which fwd; done" \
  "c2:400:for i in 1 2; do $C; TOUED_LIB=${E}FWD_HDEFER_0.so $C; done"
