#!/bin/bash
# Round 6, call 4: determinism probe of the meta-gradient step on the unit-quad layouts; BWD_DGQ timing
B="python tools/bench_gru.py --which bwd"
E=$(pwd)/to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r06t4 \
  "det:200:python tools/det_meta.py dense 4 2 && python tools/det_meta.py tabular 8 5 && TOUED_LIB=${E}head.so python tools/det_meta.py dense 4 2" \
  "dgq:200:for i in 1 2; do $B; TOUED_LIB=${E}BWD_DGQ_1.so $B; done"
