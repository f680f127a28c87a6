#!/bin/bash
# Round 4 (i): V(obs) loaded inside the A2C env chain and the restrict-qualified GAE scan: parity, stamps, C3 bench
E=to-ued_amd/exp/libtoued_
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_steps.sh r04i \
  "plr:400:$T tests/test_gpu_plr.py" \
  "fine:200:TOUED_LIB=${E}A2C_STAMPS_1_A2C_STAMPS_FINE_1.so python tools/a2c_stamps.py" \
  "c3:300:python bench.py --no_cpu_baseline --workloads c3 --steps 3"
