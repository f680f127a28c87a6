#!/bin/bash
# Round 6, call 15: the sorted-row kernels reading the per-agent time rows once per block (LDS) and HvpOp's gathers
# off scalar bases in two stages: bit identity against the previous commit's library (two head dumps calibrate
# the scratch buffers), the phase stamps, and the C2 bench against the previous commit
H=$(pwd)/to-ued_amd/exp/libtoued_head.so
E=$(pwd)/to-ued_amd/exp/libtoued_
O=gpurun_out/r06t15
D="python tools/ab_dump.py"
C="python bench.py --workloads none --no_cpu_baseline --steps 10"
bash tools/gpu_steps.sh r06t15 \
  "dump:300:TOUED_LIB=$H $D dump $O/h1.pt dense 64 5 && TOUED_LIB=$H $D dump $O/h2.pt dense 64 5 && $D dump $O/n.pt dense 64 5 && TOUED_LIB=$H $D dump $O/hs.pt sparse 64 5 && $D dump $O/ns.pt sparse 64 5" \
  "cmp:120:$D compare $O/h1.pt $O/h2.pt; $D compare $O/h1.pt $O/n.pt; $D compare $O/hs.pt $O/ns.pt; rm -f $O/*.pt" \
  "rst:300:TOUED_LIB=${E}ROWS_STAMPS_1.so python tools/rows_stamps.py" \
  "c2:400:$C && TOUED_LIB=$H $C && $C"
