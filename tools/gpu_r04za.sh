#!/bin/bash
# Round 4 (za): A2C chain with one-wave env workers as the default: A2C tests, C3 bench, regret-round trace
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_steps.sh r04za \
  "plr:400:$T tests/test_gpu_plr.py" \
  "c3:300:python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "round:300:bash tools/trace_round.sh r04za"
