#!/bin/bash
# Round 6, call 35: the forward with only the head-partial fold re-deriving its lane (FWD_XOR32=1: no spilled-index
# reload, and so no drain of the save stores, in the middle of the gate maths; FWD_LANEB off): bit identity
# against FWD_XOR32=0 (default; the variant library is FWD_XOR32_1), the forward (C2 and C4 instances) A/B, the C2 bench
E=$(pwd)/to-ued_amd/exp/libtoued_
O=gpurun_out/r06t35
D="python tools/ab_dump.py"
B="python tools/bench_gru.py --which fwd"
M="python tools/bench_fwd_multi.py"
C="python bench.py --workloads none --no_cpu_baseline --steps 10"
bash tools/gpu_steps.sh r06t35 \
  "dump:300:TOUED_LIB=${E}FWD_XOR32_1.so $D dump $O/h.pt dense 64 5 && $D dump $O/n.pt dense 64 5" \
  "cmp:120:$D compare $O/h.pt $O/n.pt; rm -f $O/*.pt" \
  "ab:300:for i in 1 2 3; do $B; TOUED_LIB=${E}FWD_XOR32_1.so $B; done" \
  "c4k:200:for i in 1 2; do $M; TOUED_LIB=${E}FWD_XOR32_1.so $M; done" \
  "c2:400:$C && TOUED_LIB=${E}FWD_XOR32_1.so $C && $C && TOUED_LIB=${E}FWD_XOR32_1.so $C"
