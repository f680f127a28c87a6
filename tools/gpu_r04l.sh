#!/bin/bash
# Round 4 (l): full suite, smoke, bench (all workloads, CPU baselines), step trace and profiles of the current defaults
bash tools/gpu_steps.sh r04l \
  "gputest:900:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:500:python bench.py" \
  "bench2:300:python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "trace:300:bash tools/trace_step.sh r04l" \
  "prof:900:bash tools/profile.sh r04l"
