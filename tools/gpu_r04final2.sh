#!/bin/bash
# Round 4 (final 2, after the eval table): the full suite, smoke, the default bench (all workloads, CPU baselines) and a regret-round trace of
# the final tree
bash tools/gpu_steps.sh r04final2 \
  "gputest:700:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:500:python bench.py" \
  "round:300:bash tools/trace_round.sh r04final2"
