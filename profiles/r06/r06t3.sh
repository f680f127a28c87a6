#!/bin/bash
# Round 6, call 3: the saves in unit-quad blocks (forward 16-byte stores, backward loads without transposes, the
# reduction's A staging with a lane-quad transpose): the -m gpu suite, then the kernels and the C2 bench against the
# previous commit's library (exp/libtoued_head.so)
B="python tools/bench_gru.py --which both"
H=$(pwd)/to-ued_amd/exp/libtoued_head.so
bash tools/gpu_steps.sh r06t3 \
  "suite:900:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15" \
  "ab:300:for i in 1 2 3; do $B; TOUED_LIB=$H $B; done" \
  "c2:400:python bench.py --workloads none --no_cpu_baseline --steps 10 && TOUED_LIB=$H python bench.py --workloads none --no_cpu_baseline --steps 10 && python bench.py --workloads none --no_cpu_baseline --steps 10"
