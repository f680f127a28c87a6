#!/bin/bash
# Round 4 (r): the C3 regret round's timeline and the A2C chain's fine stamps under the no-ramp default
E=to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r04r \
  "fine:200:TOUED_LIB=${E}A2C_STAMPS_1_A2C_STAMPS_FINE_1.so python tools/a2c_stamps.py" \
  "round:300:bash tools/trace_round.sh r04r"
