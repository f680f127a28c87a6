#!/bin/bash
# Round 4 (zc): the self-drawing A2C chain with one key-chain wave feeding two draw waves through LDS
# (A2C_SELF_SPLIT, TOUED_A2C_SELF=1): A2C tests (both chain modes), C3 A/B against the default, regret-round trace
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_steps.sh r04zc \
  "plr:400:$T tests/test_gpu_plr.py" \
  "c3_self:300:TOUED_A2C_SELF=1 python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_old:300:python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_self2:300:TOUED_A2C_SELF=1 python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "round:300:TOUED_A2C_SELF=1 bash tools/trace_round.sh r04zc"
