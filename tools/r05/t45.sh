#!/bin/bash
# Round 5: the C2 train rollout's env chain in 64- / 128-thread workgroups (TOUED_TRAIN_ENV_BLOCK) against 256: C2 A/B
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t45 \
  "par:300:TOUED_TRAIN_ENV_BLOCK=64 python -u -m pytest tests/test_gpu_env.py -q -x --timeout 300 --timeout-method thread -k 'train_rollout'" \
  "c2:600:$C && TOUED_TRAIN_ENV_BLOCK=64 $C && TOUED_TRAIN_ENV_BLOCK=128 $C && $C && TOUED_TRAIN_ENV_BLOCK=64 $C && TOUED_TRAIN_ENV_BLOCK=128 $C"
