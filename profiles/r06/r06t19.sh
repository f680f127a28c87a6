#!/bin/bash
# Round 6, call 19: the fused reverse-step kernel at 96 VGPRs (agent.hip without the SLP vectoriser, 5 waves per
# SIMD: variant noslp5) -- do the key chain's waves still keep 64 of its blocks a round late?  Block spans, bit
# identity against the previous commit's library, the C2 bench
H=$(pwd)/to-ued_amd/exp/libtoued_head.so
E=$(pwd)/to-ued_amd/exp/libtoued_
O=gpurun_out/r06t19
D="python tools/ab_dump.py"
C="python bench.py --workloads none --no_cpu_baseline --steps 10"
bash tools/gpu_steps.sh r06t19 \
  "rst:300:TOUED_LIB=${E}noslp5_st.so python tools/rows_stamps.py" \
  "dump:300:TOUED_LIB=$H $D dump $O/h.pt dense 64 5 && TOUED_LIB=${E}noslp5.so $D dump $O/n.pt dense 64 5" \
  "cmp:120:$D compare $O/h.pt $O/n.pt; rm -f $O/*.pt" \
  "c2:500:$C && TOUED_LIB=${E}noslp5.so $C && $C && TOUED_LIB=${E}noslp5.so $C"
