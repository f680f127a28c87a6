#!/bin/bash
# Round 5: h_in in slab blocks too: the whole -m gpu suite, smoke, the C2 step, forward and backward alone
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t27 \
  "gputest:700:python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread" \
  "smoke:150:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "c2:300:$C && $C" \
  "gru:200:python tools/bench_gru.py --which fwd && python tools/bench_gru.py --which bwd && python tools/bench_gru.py --which bwd"
