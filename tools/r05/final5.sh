#!/bin/bash
# Round 5 (final, with the eval prep after the last forward): the full -m gpu suite, smoke, the default bench
bash tools/gpu_steps.sh r05final5 \
  "gputest:900:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "smoke:150:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py"
