#!/bin/bash
# Round 5: DG in slab blocks (fused backward -> toued_wgrad_bfp_slab): parity, the C2 step, the backward, traffic
export TMPDIR=/tmp
O=$(pwd)/gpurun_out/r05t25
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t25 \
  "par:400:python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_fullsize.py tests/test_gpu_meta.py -q -x --timeout 200 --timeout-method thread" \
  "c2:300:$C && $C" \
  "bwd:200:python tools/bench_gru.py --which bwd && python tools/bench_gru.py --which bwd" \
  "pmc:150:timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc -o run -- python3 bench.py --steps 1 --warmup 1 --no_cpu_baseline --workloads none" \
  "sum:60:python tools/pmc_kernel.py FETCH_SIZE k_wgrad $O/pmc && find $O -name '*.db' -delete"
