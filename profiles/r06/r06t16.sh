#!/bin/bash
# Round 6, call 16: the fused reverse-step kernel (k_rows_sorted2) under 120 VGPRs, so that two of its blocks and a
# key-chain wave share a CU: the thread index laundered per body, HvpOp's time-row sums after its sample loop, and
# (variant noslp) agent.hip without the SLP vectoriser.  Bit identity against the previous commit, phase stamps and
# block spans, and the C2 bench
H=$(pwd)/to-ued_amd/exp/libtoued_head.so
E=$(pwd)/to-ued_amd/exp/libtoued_
O=gpurun_out/r06t16
D="python tools/ab_dump.py"
C="python bench.py --workloads none --no_cpu_baseline --steps 10"
bash tools/gpu_steps.sh r06t16 \
  "dump:300:TOUED_LIB=$H $D dump $O/h.pt dense 64 5 && $D dump $O/n.pt dense 64 5 && TOUED_LIB=${E}noslp.so $D dump $O/s.pt dense 64 5 && TOUED_LIB=$H $D dump $O/hs.pt sparse 64 5 && TOUED_LIB=${E}noslp.so $D dump $O/ss.pt sparse 64 5" \
  "cmp:120:$D compare $O/h.pt $O/n.pt; $D compare $O/h.pt $O/s.pt; $D compare $O/hs.pt $O/ss.pt; rm -f $O/*.pt" \
  "rst:300:TOUED_LIB=${E}ROWS_STAMPS_1.so python tools/rows_stamps.py && TOUED_LIB=${E}noslp_st.so python tools/rows_stamps.py" \
  "c2:500:$C && TOUED_LIB=${E}noslp.so $C && TOUED_LIB=$H $C && TOUED_LIB=${E}noslp.so $C && $C"
