#!/bin/bash
# Round 5 timing study: the sorted row kernels without their sort (ROWS_TNOSORT=1, wrong results) -- the sort's share
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r05t51 \
  "ns:400:TOUED_LIB=${E}ROWS_TNOSORT_1.so bash tools/trace_step.sh r05ns" \
  "s:400:bash tools/trace_step.sh r05s"
