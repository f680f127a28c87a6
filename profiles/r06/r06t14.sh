#!/bin/bash
# Round 6, call 14: phase stamps of the per-agent sorted-row kernels (inner update and reverse step) in a C2 step
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r06t14 "rst:300:TOUED_LIB=${E}ROWS_STAMPS_1.so python tools/rows_stamps.py"
