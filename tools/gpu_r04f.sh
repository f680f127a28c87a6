#!/bin/bash
# Round 4 (f): the med3 bitonic sort (parity, A2C stamps and C3/C2 A/B against SORT_MED3=0), then the
# TOUED_EVAL_KEYS_EARLY, H3_B_AUX=2 and FWD_AUG32=1 A/B runs of r04e.
B="python bench.py --no_cpu_baseline --workloads none --steps 10"
X=to-ued_amd/exp
bash tools/gpu_steps.sh r04f \
  "sort:120:python -u -m pytest tests/test_gpu_sort.py -x -q --timeout 60 --timeout-method thread" \
  "parA:400:python -u -m pytest tests/test_gpu_env.py tests/test_gpu_plr.py tests/test_gpu_meta.py -x -q --timeout 120 --timeout-method thread" \
  "st1:200:TOUED_LIB=$X/libtoued_A2C_STAMPS_1.so python tools/a2c_stamps.py" \
  "st0:200:TOUED_LIB=$X/libtoued_A2C_STAMPS_1_SORT_MED3_0.so python tools/a2c_stamps.py" \
  "c3n:300:python bench.py --no_cpu_baseline --workloads c3 --steps 3" \
  "c3o:300:TOUED_LIB=$X/libtoued_SORT_MED3_0.so python bench.py --no_cpu_baseline --workloads c3 --steps 3" \
  "e0:200:TOUED_EVAL_KEYS_EARLY=0 $B && TOUED_EVAL_KEYS_EARLY=0 $B" \
  "e1:200:TOUED_EVAL_KEYS_EARLY=1 $B && TOUED_EVAL_KEYS_EARLY=1 $B" \
  "o0:200:TOUED_EVAL_KEYS_EARLY=0 TOUED_LIB=$X/libtoued_SORT_MED3_0.so $B" \
  "n1:200:TOUED_EVAL_KEYS_EARLY=1 TOUED_LIB=$X/libtoued_H3_B_AUX_2.so $B && TOUED_EVAL_KEYS_EARLY=1 TOUED_LIB=$X/libtoued_H3_B_AUX_2.so $B" \
  "par:400:TOUED_EVAL_KEYS_EARLY=1 python -u -m pytest tests/test_gpu_curve.py tests/test_gpu_c5.py -x -q --timeout 120 --timeout-method thread" \
  "trace:300:TOUED_EVAL_KEYS_EARLY=1 bash tools/trace_step.sh r04f" && \
bash tools/gpu_steps.sh r04f \
  "c4a:300:python bench.py --no_cpu_baseline --workloads c4 --steps 4" \
  "c4b:300:TOUED_LIB=$X/libtoued_FWD_AUG32_1.so python bench.py --no_cpu_baseline --workloads c4 --steps 4" \
  "parC4:400:TOUED_LIB=$X/libtoued_FWD_AUG32_1.so python -u -m pytest tests/test_gpu_es.py tests/test_gpu_es_curve.py -x -q --timeout 120 --timeout-method thread"
