#!/bin/bash
# Round 5: h_in in slab blocks vs rows (HIN_SLAB=0 variant), same box, interleaved
E=$(pwd)/to-ued_amd/exp/libtoued_
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t29 \
  "c2:500:for i in 1 2 3; do $C; TOUED_LIB=${E}HIN_SLAB_0.so $C; done" \
  "gru:300:for i in 1 2; do python tools/bench_gru.py --which bwd; TOUED_LIB=${E}HIN_SLAB_0.so python tools/bench_gru.py --which bwd; python tools/bench_gru.py --which fwd; TOUED_LIB=${E}HIN_SLAB_0.so python tools/bench_gru.py --which fwd; done"
