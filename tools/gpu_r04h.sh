#!/bin/bash
# Round 4 (h): where the A2C chain's GAE phase and env chain spend their cycles (fine stamps; the env chain without
# its row gathers, timing only)
E=to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r04h \
  "fine:200:TOUED_LIB=${E}A2C_STAMPS_1_A2C_STAMPS_FINE_1.so python tools/a2c_stamps.py" \
  "nog:200:TOUED_LIB=${E}A2C_STAMPS_1_A2C_NOGATHER_1.so python tools/a2c_stamps.py" \
  "st:200:TOUED_LIB=${E}A2C_STAMPS_1.so python tools/a2c_stamps.py"
