#!/bin/bash
# Round 4 (t): every chunk's A2C key chains made up front (TOUED_A2C_KEYS_AHEAD=1, default) instead of beside the chain
# launches: A2C tests, C3 A/B, regret-round trace
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_steps.sh r04t \
  "plr:400:$T tests/test_gpu_plr.py" \
  "c3_ahead:300:python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_old:300:TOUED_A2C_KEYS_AHEAD=0 python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_ahead2:300:python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "round:300:bash tools/trace_round.sh r04t"
