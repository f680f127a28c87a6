#!/bin/bash
# Round 4 (o): C3 regret-round knobs: the chunk ramp, the chain's wave priority, the eval-draw split
E=to-ued_amd/exp/libtoued_
C="python bench.py --no_cpu_baseline --workloads c3 --steps 4"
bash tools/gpu_steps.sh r04o \
  "d0:200:$C" \
  "noramp:200:TOUED_A2C_RAMP=0 $C" \
  "p1:200:TOUED_LIB=${E}A2C_PRIO_1.so $C" \
  "p0:200:TOUED_LIB=${E}A2C_PRIO_0.so $C" \
  "nosplit:200:TOUED_REGRET_SPLIT_EVAL=0 $C" \
  "d1:200:$C"
