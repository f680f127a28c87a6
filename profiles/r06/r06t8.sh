#!/bin/bash
# Round 6, call 8: r / z / hn saves in unit-quad blocks (b128 + s_nop 1): the -m gpu suite, smoke, C2 bench vs the
# previous commit
H=$(pwd)/to-ued_amd/exp/libtoued_head.so
bash tools/gpu_steps.sh r06t8 \
  "suite:1000:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15" \
  "smoke:150:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "c2:400:python bench.py --workloads none --no_cpu_baseline --steps 10 && TOUED_LIB=$H python bench.py --workloads none --no_cpu_baseline --steps 10 && python bench.py --workloads none --no_cpu_baseline --steps 10"
