#!/bin/bash
# Round 5: kernel traces with and without the phase-1 warm-up (per-kernel times of the sorted row kernels)
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r05t49 \
  "w0:400:TOUED_LIB=${E}ROWS_WARM_0.so bash tools/trace_step.sh r05w0" \
  "w1:400:bash tools/trace_step.sh r05w1"
