#!/bin/bash
# Round 4 (j): A2C parity after the V-gather revert + restrict GAE scan, fine stamps; the reverse agent loop's
# k_rows_sorted at wave priority 3 beside eval_agent's key chain (ROWS_PRIO) against the default
E=to-ued_amd/exp/libtoued_
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
B="python bench.py --no_cpu_baseline --workloads none --steps 10"
bash tools/gpu_steps.sh r04j \
  "plr:400:$T tests/test_gpu_plr.py" \
  "fine:200:TOUED_LIB=${E}A2C_STAMPS_1_A2C_STAMPS_FINE_1.so python tools/a2c_stamps.py" \
  "p0:200:$B && $B" \
  "p3:200:TOUED_LIB=${E}ROWS_PRIO_3.so $B && TOUED_LIB=${E}ROWS_PRIO_3.so $B" \
  "p0b:200:$B" \
  "tr3:300:TOUED_LIB=${E}ROWS_PRIO_3.so bash tools/trace_step.sh r04j_p3"
