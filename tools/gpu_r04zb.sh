#!/bin/bash
# Round 4 (zb): the self-drawing A2C chain (toued_a2c_chain_self, TOUED_A2C_SELF=1): A2C tests (both chain modes),
# C3 A/B against the chunked chain with the draws pass beside it, regret-round trace; then the full suite, smoke and
# the default bench of the current tree
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_steps.sh r04zb \
  "plr:400:$T tests/test_gpu_plr.py" \
  "c3_self:300:TOUED_A2C_SELF=1 python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_old:300:python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_self2:300:TOUED_A2C_SELF=1 python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "round:300:TOUED_A2C_SELF=1 bash tools/trace_round.sh r04zb" \
  "gputest:900:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:500:python bench.py"
