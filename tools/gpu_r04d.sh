#!/bin/bash
# backward DG-store placement variants (two timings each), stamps, then the full suite and smoke of the default
B="python tools/bench_gru.py --which bwd"
E=to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r04d \
  "v0:120:$B && $B" \
  "s1:120:TOUED_LIB=${E}BWD_STMEM_1.so $B && TOUED_LIB=${E}BWD_STMEM_1.so $B" \
  "s2:120:TOUED_LIB=${E}BWD_STMEM_2.so $B && TOUED_LIB=${E}BWD_STMEM_2.so $B" \
  "s1n4:120:TOUED_LIB=${E}BWD_STMEM_1_BWD_NR_4.so $B && TOUED_LIB=${E}BWD_STMEM_1_BWD_NR_4.so $B" \
  "s2n4:120:TOUED_LIB=${E}BWD_STMEM_2_BWD_NR_4.so $B && TOUED_LIB=${E}BWD_STMEM_2_BWD_NR_4.so $B" \
  "v0b:120:$B && $B" \
  "stamps:120:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "stamps1:120:TOUED_LIB=${E}BWD_STMEM_1_BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "gputest:900:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:400:python bench.py" \
  "trace:300:bash tools/trace_step.sh r04d"
