#!/bin/bash
# variant timings of the fused backward first (two runs each), stamps, a parity pass of the early-scale variant, then
# the suite, smoke and profiles of the default library
B="python tools/bench_gru.py --which bwd"
E=to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r04c \
  "v0:120:$B && $B" \
  "v1:120:TOUED_LIB=${E}BWD_DWORD_LD_1.so $B && TOUED_LIB=${E}BWD_DWORD_LD_1.so $B" \
  "v2:120:TOUED_LIB=${E}BWD_DWORD_LD_1_BWD_NR_4.so $B && TOUED_LIB=${E}BWD_DWORD_LD_1_BWD_NR_4.so $B" \
  "v3:120:TOUED_LIB=${E}BWD_NR_4.so $B && TOUED_LIB=${E}BWD_NR_4.so $B" \
  "v4:120:TOUED_LIB=${E}BWD_EARLY_1.so $B && TOUED_LIB=${E}BWD_EARLY_1.so $B" \
  "v5:120:TOUED_LIB=${E}BWD_EARLY_1_BWD_DWORD_LD_1.so $B && TOUED_LIB=${E}BWD_EARLY_1_BWD_DWORD_LD_1.so $B" \
  "v6:120:TOUED_LIB=${E}BWD_EARLY_1_BWD_DWORD_LD_1_BWD_NR_4.so $B && TOUED_LIB=${E}BWD_EARLY_1_BWD_DWORD_LD_1_BWD_NR_4.so $B" \
  "f0:120:python tools/bench_gru.py --which fwd && python tools/bench_gru.py --which fwd" \
  "f1:120:TOUED_LIB=${E}FWD_LAZY_1.so python tools/bench_gru.py --which fwd && TOUED_LIB=${E}FWD_LAZY_1.so python tools/bench_gru.py --which fwd" \
  "parF:300:TOUED_LIB=${E}FWD_LAZY_1.so python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_es.py -x -q --timeout 120 --timeout-method thread" \
  "stamps:120:TOUED_LIB=${E}BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "stamps1:120:TOUED_LIB=${E}BWD_DWORD_LD_1_BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "stamps5:120:TOUED_LIB=${E}BWD_EARLY_1_BWD_DWORD_LD_1_BWD_STAMPS_1.so python tools/bwd_stamps.py" \
  "par5:300:TOUED_LIB=${E}BWD_EARLY_1_BWD_DWORD_LD_1.so python -u -m pytest tests/test_gpu_meta.py -x -q --timeout 120 --timeout-method thread" \
  "gputest:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "prof:900:bash tools/profile.sh r04c"
