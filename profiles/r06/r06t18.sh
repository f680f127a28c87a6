#!/bin/bash
# Round 6, call 18: why 64 blocks of every reverse-step launch start a round late -- block spans with eval_agent's key
# chain in 256-thread workgroups (16 instead of 64) and with the key chain after the backward (nothing beside the
# reverse loop), and the C2 step with the 256-thread key chain
E=$(pwd)/to-ued_amd/exp/libtoued_
C="python bench.py --workloads none --no_cpu_baseline --steps 10"
R="python tools/rows_stamps.py"
bash tools/gpu_steps.sh r06t18 \
  "kb256:300:TOUED_EVAL_KEYS_BLOCK=256 TOUED_LIB=${E}ROWS_STAMPS_1.so $R" \
  "early0:300:TOUED_EVAL_KEYS_EARLY=0 TOUED_LIB=${E}ROWS_STAMPS_1.so $R" \
  "c2:500:$C && TOUED_EVAL_KEYS_BLOCK=256 $C && $C && TOUED_EVAL_KEYS_BLOCK=256 $C"
