#!/bin/bash
# Round 5 (final): the full suite, smoke, the default bench (all workloads, CPU baselines); profiles in a second call
# (bash tools/profile.sh r05)
bash tools/gpu_steps.sh r05final \
  "gputest:700:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "smoke:150:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py"
