#!/bin/bash
# Round 4 (u): the meta-step prologue stream (key splits, level sampler, train draws beside the main reduction):
# meta / curve / sampler tests, C2 A/B against TOUED_PROLOGUE_OVERLAP=0, step trace
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh r04u \
  "tests:600:$T tests/test_gpu_curve.py tests/test_gpu_meta.py tests/test_gpu_c5.py tests/test_gpu_sampler.py" \
  "c2_on:200:python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "c2_off:200:TOUED_PROLOGUE_OVERLAP=0 python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "c2_on2:200:python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "c2_off2:200:TOUED_PROLOGUE_OVERLAP=0 python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "trace:300:bash tools/trace_step.sh r04u"
