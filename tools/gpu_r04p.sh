#!/bin/bash
# Round 4 (p): C3 draw-chunk ramps and how early the eval draws are enqueued
C="python bench.py --no_cpu_baseline --workloads c3 --steps 4"
bash tools/gpu_steps.sh r04p \
  "r1:200:$C" \
  "r0:200:TOUED_A2C_RAMP=0 $C" \
  "r16:200:TOUED_A2C_RAMP=16 $C" \
  "r816:200:TOUED_A2C_RAMP=8,16 $C" \
  "r1224:200:TOUED_A2C_RAMP=12,24 $C" \
  "r0e3:200:TOUED_A2C_RAMP=0 TOUED_A2C_EV_AHEAD=3 $C" \
  "r0e4:200:TOUED_A2C_RAMP=0 TOUED_A2C_EV_AHEAD=4 $C" \
  "r0b:200:TOUED_A2C_RAMP=0 $C"
