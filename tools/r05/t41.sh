#!/bin/bash
# Round 5: this session's C2 step changes all off (launch-per-op paths, copy-back history, k_embed_bwd) against the
# default, interleaved, and a kernel trace of the default
E=$(pwd)/to-ued_amd/exp/libtoued_
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
O="TOUED_LIB=${E}EMBED_V_1.so TOUED_REVERSE_PAIR=0 TOUED_SAMPLE_FUSED=0 TOUED_STEP_ENTROPY=0 TOUED_HIST_RING=0 TOUED_PACK_SIDE=0"
bash tools/gpu_steps.sh r05t41 \
  "c2:600:$O $C && $C && $O $C && $C && $O $C && $C" \
  "trace:400:bash tools/trace_step.sh r05c"
