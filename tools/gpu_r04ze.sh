#!/bin/bash
# Round 4 (ze): eval_agent's env chain with a per-wave transition table in LDS (k_eval_returns<TBL>, W % 64 == 0):
# env + A2C tests, C3 A/B against TOUED_EVAL_TBL=0, C4
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_steps.sh r04ze \
  "env:400:$T tests/test_gpu_env.py tests/test_gpu_plr.py" \
  "c3_tbl:300:python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_off:300:TOUED_EVAL_TBL=0 python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_tbl2:300:python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_off2:300:TOUED_EVAL_TBL=0 python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "round:300:bash tools/trace_round.sh r04ze"
