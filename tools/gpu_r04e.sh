#!/bin/bash
# eval_agent key chain + draws beside the reverse agent loop (TOUED_EVAL_KEYS_EARLY) against after the backward
B="python bench.py --no_cpu_baseline --workloads none --steps 10"
bash tools/gpu_steps.sh r04e \
  "e0:200:TOUED_EVAL_KEYS_EARLY=0 $B && TOUED_EVAL_KEYS_EARLY=0 $B" \
  "e1:200:TOUED_EVAL_KEYS_EARLY=1 $B && TOUED_EVAL_KEYS_EARLY=1 $B" \
  "e0b:200:TOUED_EVAL_KEYS_EARLY=0 $B" \
  "n1:200:TOUED_EVAL_KEYS_EARLY=1 TOUED_LIB=to-ued_amd/exp/libtoued_H3_B_AUX_2.so $B && TOUED_EVAL_KEYS_EARLY=1 TOUED_LIB=to-ued_amd/exp/libtoued_H3_B_AUX_2.so $B" \
  "e1b:200:TOUED_EVAL_KEYS_EARLY=1 $B" \
  "par:400:TOUED_EVAL_KEYS_EARLY=1 python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_curve.py tests/test_gpu_c5.py -x -q --timeout 120 --timeout-method thread" \
  "trace:300:TOUED_EVAL_KEYS_EARLY=1 bash tools/trace_step.sh r04e" \
  "trace2:300:TOUED_EVAL_KEYS_EARLY=1 TOUED_LIB=to-ued_amd/exp/libtoued_H3_B_AUX_2.so bash tools/trace_step.sh r04e_nt" && \
bash tools/gpu_steps.sh r04e \
  "c4a:300:python bench.py --no_cpu_baseline --workloads c4 --steps 4" \
  "c4b:300:TOUED_LIB=to-ued_amd/exp/libtoued_FWD_AUG32_1.so python bench.py --no_cpu_baseline --workloads c4 --steps 4" \
  "parC4:400:TOUED_LIB=to-ued_amd/exp/libtoued_FWD_AUG32_1.so python -u -m pytest tests/test_gpu_es.py tests/test_gpu_es_curve.py -x -q --timeout 120 --timeout-method thread"
