#!/bin/bash
# Round 5 (final, slab layouts): the full suite, smoke, the default bench (all workloads, CPU baselines)
bash tools/gpu_steps.sh r05final2 \
  "gputest:700:python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread" \
  "smoke:150:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py"
