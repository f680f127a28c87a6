#!/bin/bash
# Round 5: eval_agent's key chain workgroup size with the chain now after the last forward (TOUED_EVAL_KEYS_BLOCK 64
# default = one wave per workgroup, 128, 256): C2 A/B
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t52 \
  "c2:700:$C && TOUED_EVAL_KEYS_BLOCK=256 $C && TOUED_EVAL_KEYS_BLOCK=128 $C && $C && TOUED_EVAL_KEYS_BLOCK=256 $C && TOUED_EVAL_KEYS_BLOCK=128 $C"
