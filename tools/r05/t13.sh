#!/bin/bash
# Round 5: k_wgrad_h3 B loads non-temporal (H3_B_AUX) alone and in the C2 step, with its FETCH_SIZE; the forward's
# lead-load order (ring before x vs the round-4 x first)
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
F="python tools/bench_gru.py --which fwd"
export TMPDIR=/tmp
P="timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -o run -- python3 bench.py --steps 1 --warmup 1 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t13 \
  "wg:300:for i in 1 2; do python tools/bench_wgrad.py; TOUED_LIB=${E}H3_B_AUX_2.so python tools/bench_wgrad.py; TOUED_LIB=${E}H3_B_AUX_1.so python tools/bench_wgrad.py; done" \
  "fwd:200:for i in 1 2; do $F; TOUED_LIB=${E}FWD_XFIRST_1.so $F; done" \
  "c2:400:for i in 1 2; do $B; TOUED_LIB=${E}H3_B_AUX_2.so $B; TOUED_LIB=${E}H3_B_AUX_1.so $B; done" \
  "pmc0:150:$P -d $(pwd)/gpurun_out/r05t13/pmc0" \
  "pmc2:150:TOUED_LIB=${E}H3_B_AUX_2.so $P -d $(pwd)/gpurun_out/r05t13/pmc2" \
  "sum:60:python tools/pmc_kernel.py FETCH_SIZE k_ gpurun_out/r05t13/pmc0 gpurun_out/r05t13/pmc2 && find gpurun_out/r05t13 -name \"*.db\" -delete"
