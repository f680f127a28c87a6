#!/bin/bash
# Round 5: the half-row forward (k_gru_fwd6h, two 32-row workgroups per CU, TOUED_FWD_H2=1) -- parity, timing, C2 bench
F="python tools/bench_gru.py --which fwd"
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r05t11 \
  "par:400:TOUED_FWD_H2=1 python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread" \
  "fwd:300:for i in 1 2; do TOUED_FWD_H2=1 $F; $F; TOUED_FWD_H2=1 TOUED_LIB=${E}FWD_H2_RING_2.so $F; done" \
  "bench:300:TOUED_FWD_H2=1 python bench.py --no_cpu_baseline --workloads none --steps 10 && python bench.py --no_cpu_baseline --workloads none --steps 10"
