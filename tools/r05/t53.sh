#!/bin/bash
# Round 5: the key chain in 256-thread workgroups against 64 (confirmation, interleaved), and a trace at 256
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t53 \
  "c2:800:$C && TOUED_EVAL_KEYS_BLOCK=256 $C && $C && TOUED_EVAL_KEYS_BLOCK=256 $C && $C && TOUED_EVAL_KEYS_BLOCK=256 $C && $C && TOUED_EVAL_KEYS_BLOCK=256 $C" \
  "trace:400:TOUED_EVAL_KEYS_BLOCK=256 bash tools/trace_step.sh r05k256"
