#!/bin/bash
# Round 6, call 28: the final tree -- the -m gpu suite, smoke(), and the default bench (headline + C3 / C4 workloads +
# CPU baseline), as the driver runs them
bash tools/gpu_steps.sh r06t28 \
  "suite:600:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15" \
  "smoke:150:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:400:python bench.py"
