#!/bin/bash
# Round 4 (z): the A2C chain's env workers in one wave (A2C_ENV_SPREAD=0) against the four-wave spread: stamps, C3
E=to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r04z \
  "st1:200:TOUED_LIB=${E}A2C_STAMPS_1_A2C_STAMPS_FINE_1.so python tools/a2c_stamps.py" \
  "st0:200:TOUED_LIB=${E}A2C_STAMPS_1_A2C_STAMPS_FINE_1_A2C_ENV_SPREAD_0.so python tools/a2c_stamps.py" \
  "c3_1:300:python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_0:300:TOUED_LIB=${E}A2C_ENV_SPREAD_0.so python bench.py --no_cpu_baseline --workloads c3 --steps 4"
