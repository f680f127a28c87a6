#!/bin/bash
# Round 6, call 11: eval_agent's env chain alone (TOUED_EVAL_ALONE=1: the main reduction after it, on every CU) -- a
# C2 kernel trace -- to split its 3.4 ms beside the reduction into its own latency and the reduction's interference
bash tools/gpu_steps.sh r06t11 \
  "trace:400:TOUED_EVAL_ALONE=1 bash tools/trace_step.sh r06t11"
