#!/bin/bash
# Round 5: k_wgrad_h3 (two-slab B ring) with B non-temporal: C2 step time and FETCH_SIZE per launch
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
export TMPDIR=/tmp
O=$(pwd)/gpurun_out/r05t21
P="rocprofv3 --pmc FETCH_SIZE --kernel-trace"
Q="-- python3 bench.py --steps 1 --warmup 1 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t21 \
  "c2:400:for i in 1 2; do $B; TOUED_LIB=${E}H3_B_AUX_2.so $B; done" \
  "pmc0:150:timeout -s KILL 120 $P -d $O/pmc0 -o run $Q" \
  "pmc2:150:TOUED_LIB=${E}H3_B_AUX_2.so timeout -s KILL 120 $P -d $O/pmc2 -o run $Q" \
  "sum:60:python tools/pmc_kernel.py FETCH_SIZE k_wgrad $O/pmc0 $O/pmc2 && find $O -name '*.db' -delete"
