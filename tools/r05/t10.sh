#!/bin/bash
# Round 5: backward memory-part issue priority; eval_agent's env chain row-gather variants beside the reduction
B="python tools/bench_gru.py --which bwd"
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r05t10 \
  "ab:300:for i in 1 2; do $B; TOUED_LIB=${E}BWD_MPRIO_1.so $B; TOUED_LIB=${E}BWD_MPRIO_2.so $B; done" \
  "st:200:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py && TOUED_LIB=${E}BWD_MPRIO_1_BWD_STAMPS_1.so python tools/bwd_stamps.py && TOUED_LIB=${E}BWD_MPRIO_2_BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "par:200:TOUED_LIB=${E}EVAL_CHOSEN_ROW_2.so python -u -m pytest tests/test_gpu_env.py -q -k eval --timeout 120 --timeout-method thread" \
  "tr0:200:bash tools/trace_step.sh r05t10_cr1" \
  "tr1:200:TOUED_LIB=${E}EVAL_CHOSEN_ROW_0.so bash tools/trace_step.sh r05t10_cr0" \
  "tr2:200:TOUED_LIB=${E}EVAL_CHOSEN_ROW_2.so bash tools/trace_step.sh r05t10_cr2"
F="python tools/bench_gru.py --which fwd"
bash tools/gpu_steps.sh r05t10b \
  "fwd:300:for i in 1 2; do $F; TOUED_LIB=${E}FWD_NOSAVE_1.so $F; TOUED_LIB=${E}FWD_NOSAVE_2.so $F; TOUED_LIB=${E}FWD_ST16T_2.so $F; done"
