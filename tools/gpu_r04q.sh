#!/bin/bash
# Round 4 (q): the A2C tests and C3 with the no-ramp chunking default
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_steps.sh r04q \
  "plr:400:$T tests/test_gpu_plr.py" \
  "c3:300:python bench.py --no_cpu_baseline --workloads c3 --steps 4"
