#!/bin/bash
# Round 4 (k): the A2C GAE statistics in wave 0 (W <= 64): parity, fine stamps, C3 bench and a regret-round trace;
# C2 with ROWS_PRIO=3 as the default
E=to-ued_amd/exp/libtoued_
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_steps.sh r04k \
  "plr:400:$T tests/test_gpu_plr.py" \
  "fine:200:TOUED_LIB=${E}A2C_STAMPS_1_A2C_STAMPS_FINE_1.so python tools/a2c_stamps.py" \
  "c3:300:python bench.py --no_cpu_baseline --workloads c3 --steps 3" \
  "c2:200:python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "round:300:bash tools/trace_round.sh r04k"
