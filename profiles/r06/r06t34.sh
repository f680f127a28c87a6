#!/bin/bash
# Round 6, call 34: the forward without register spills (FWD_XOR32=1, default: the head-partial fold and the B
# fragment loads re-derive the lane index instead of reloading spilled copies -- the fold's reload waited for every
# outstanding save store in the middle of the gate maths): bit identity against FWD_XOR32=0, the forward (C2 and C4
# instances) A/B, stamps, the C2 bench
E=$(pwd)/to-ued_amd/exp/libtoued_
O=gpurun_out/r06t34
D="python tools/ab_dump.py"
B="python tools/bench_gru.py --which fwd"
M="python tools/bench_fwd_multi.py"
C="python bench.py --workloads none --no_cpu_baseline --steps 10"
bash tools/gpu_steps.sh r06t34 \
  "dump:300:TOUED_LIB=${E}FWD_XOR32_0.so $D dump $O/h.pt dense 64 5 && $D dump $O/n.pt dense 64 5" \
  "cmp:120:$D compare $O/h.pt $O/n.pt; rm -f $O/*.pt" \
  "st:200:TOUED_LIB=${E}FWD_STAMPS_1.so python tools/fwd_stamps.py --gm" \
  "ab:300:for i in 1 2 3; do $B; TOUED_LIB=${E}FWD_XOR32_0.so $B; done" \
  "c4k:200:for i in 1 2; do $M; TOUED_LIB=${E}FWD_XOR32_0.so $M; done" \
  "c2:400:$C && TOUED_LIB=${E}FWD_XOR32_0.so $C && $C && TOUED_LIB=${E}FWD_XOR32_0.so $C"
