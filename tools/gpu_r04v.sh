#!/bin/bash
# Round 4 (v): padded column stride of the GRU operands (TOUED_GRU_COL_PAD floats; the unpadded stride K*T*R*4 B is a
# multiple of 512 KiB): meta tests with and without the pad, C2 A/B over pads
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh r04v \
  "meta:400:$T tests/test_gpu_meta.py" \
  "meta_pad:400:TOUED_GRU_COL_PAD=64 $T tests/test_gpu_meta.py -k 'meta_step or backward or fused'" \
  "p0:200:python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "p64:200:TOUED_GRU_COL_PAD=64 python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "p32:200:TOUED_GRU_COL_PAD=32 python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "p1040:200:TOUED_GRU_COL_PAD=1040 python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "p0b:200:python bench.py --no_cpu_baseline --workloads none --steps 10" \
  "p64b:200:TOUED_GRU_COL_PAD=64 python bench.py --no_cpu_baseline --workloads none --steps 10"
