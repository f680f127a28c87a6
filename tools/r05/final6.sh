#!/bin/bash
# Round 5 (final, k_sum_rows_add fixed): the full -m gpu suite, smoke, the default bench, the profiles
bash tools/gpu_steps.sh r05final6 \
  "gputest:900:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "smoke:150:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py" \
  "prof:1000:bash tools/profile.sh r05"
