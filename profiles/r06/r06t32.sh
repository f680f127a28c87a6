#!/bin/bash
# Round 6, call 32: the forward's h_in saves as one transposed 16-byte store per lane quad (FWD_HQ=1, the same slab
# layout): bit identity of a meta-step against the default, forward timing A/B,
# the C2 bench
E=$(pwd)/to-ued_amd/exp/libtoued_
O=gpurun_out/r06t32
D="python tools/ab_dump.py"
B="python tools/bench_gru.py --which fwd"
C="python bench.py --workloads none --no_cpu_baseline --steps 10"
bash tools/gpu_steps.sh r06t32 \
  "dump:300:$D dump $O/h.pt dense 64 5 && TOUED_LIB=${E}FWD_HQ_1.so $D dump $O/n.pt dense 64 5" \
  "cmp:120:$D compare $O/h.pt $O/n.pt; rm -f $O/*.pt" \
  "ab:300:for i in 1 2 3; do $B; TOUED_LIB=${E}FWD_HQ_1.so $B; done" \
  "c2:400:$C && TOUED_LIB=${E}FWD_HQ_1.so $C && $C && TOUED_LIB=${E}FWD_HQ_1.so $C"
