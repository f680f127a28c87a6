#!/bin/bash
# Round 6, call 31: the forward's gate maths over both row tiles per element (FWD_HW=1: head weights and unscales
# read from LDS once for the two tiles): bit identity of a meta-step against the default, forward timing A/B,
# the C2 bench
E=$(pwd)/to-ued_amd/exp/libtoued_
O=gpurun_out/r06t31
D="python tools/ab_dump.py"
B="python tools/bench_gru.py --which fwd"
C="python bench.py --workloads none --no_cpu_baseline --steps 10"
bash tools/gpu_steps.sh r06t31 \
  "dump:300:$D dump $O/h.pt dense 64 5 && TOUED_LIB=${E}FWD_HW_1.so $D dump $O/n.pt dense 64 5" \
  "cmp:120:$D compare $O/h.pt $O/n.pt; rm -f $O/*.pt" \
  "st:200:TOUED_LIB=${E}FWD_HW_1_FWD_STAMPS_1.so python tools/fwd_stamps.py --gm" \
  "ab:300:for i in 1 2 3; do $B; TOUED_LIB=${E}FWD_HW_1.so $B; done" \
  "c2:400:$C && TOUED_LIB=${E}FWD_HW_1.so $C && $C && TOUED_LIB=${E}FWD_HW_1.so $C"
