#!/bin/bash
# Round 6, call 22: per-launch phase stamps of the sorted-row kernels (the inner update's phases, apart from
# k_rows_sorted<LpgLossOp>), then the -m gpu suite on the current tree
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r06t22 \
  "rst:300:TOUED_LIB=${E}ROWS_STAMPS_1.so python tools/rows_stamps.py" \
  "suite:1000:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15"
