#!/bin/bash
# Round 5: per-wave pass stamps of the backward; eval_agent's env chain variants beside the main reduction
E=to-ued_amd/exp/libtoued_
V=${E}EVAL_CHOSEN_ROW_1.so
bash tools/gpu_steps.sh r05t5 \
  "stamps:120:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py && TOUED_LIB=${E}BWD_SPREAD_0_BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "par:200:TOUED_EVAL_BLOCK=64 python -u -m pytest tests/test_gpu_env.py -q -k eval --timeout 120 --timeout-method thread && TOUED_LIB=$V python -u -m pytest tests/test_gpu_env.py -q -k eval --timeout 120 --timeout-method thread" \
  "tr0:200:bash tools/trace_step.sh r05t5_def" \
  "tr1:200:TOUED_EVAL_BLOCK=64 bash tools/trace_step.sh r05t5_b64" \
  "tr2:200:TOUED_EVAL_BLOCK=128 bash tools/trace_step.sh r05t5_b128" \
  "tr3:200:TOUED_LIB=$V bash tools/trace_step.sh r05t5_cr" \
  "tr4:200:TOUED_LIB=$V TOUED_EVAL_BLOCK=64 bash tools/trace_step.sh r05t5_crb64" \
  "bench:300:python bench.py --no_cpu_baseline --workloads none --steps 10 && TOUED_EVAL_BLOCK=64 python bench.py --no_cpu_baseline --workloads none --steps 10 && TOUED_LIB=${E}BWD_SPREAD_0.so python bench.py --no_cpu_baseline --workloads none --steps 10"
