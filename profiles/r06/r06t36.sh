#!/bin/bash
# Round 6, call 36: the final tree again (the forward's default-off spill variants added since r06t28) -- the -m gpu
# suite, smoke(), and the default bench
bash tools/gpu_steps.sh r06t36 \
  "suite:600:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15" \
  "smoke:150:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:400:python bench.py"
