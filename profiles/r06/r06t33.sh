#!/bin/bash
# Round 6, call 33: the inner update's entropy metrics with every sample's loads unconditional (clamped; the term
# stores past the end into dead LDS), so the four samples' gathers are in flight together: bit identity against the
# previous commit's library, phase stamps, the C2 bench
H=$(pwd)/to-ued_amd/exp/libtoued_head.so
E=$(pwd)/to-ued_amd/exp/libtoued_
O=gpurun_out/r06t33
D="python tools/ab_dump.py"
C="python bench.py --workloads none --no_cpu_baseline --steps 10"
bash tools/gpu_steps.sh r06t33 \
  "dump:300:TOUED_LIB=$H $D dump $O/h.pt dense 64 5 && $D dump $O/n.pt dense 64 5 && TOUED_LIB=$H $D dump $O/hs.pt sparse 64 5 && $D dump $O/ns.pt sparse 64 5" \
  "cmp:120:$D compare $O/h.pt $O/n.pt; $D compare $O/hs.pt $O/ns.pt; rm -f $O/*.pt" \
  "rst:300:TOUED_LIB=${E}ROWS_STAMPS_1.so python tools/rows_stamps.py" \
  "c2:500:$C && TOUED_LIB=$H $C && $C && TOUED_LIB=$H $C"
