#!/bin/bash
# Round 4 (g): the A2C chain's parity after the explicit-FMA fix (and, if it fails, the same test with the LDS
# transition table off to isolate it), stamps, then the full suite, smoke, bench, trace and profiles of the defaults
# (EVAL_KEYS_EARLY=1, FWD_AUG32=1, med3 sort, env-step table, fast A2C update maths)
E=to-ued_amd/exp/libtoued_
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_steps.sh r04g \
  "plr:400:$T tests/test_gpu_plr.py tests/test_gpu_sort.py || TOUED_LIB=${E}A2C_NPT_0.so $T tests/test_gpu_plr.py -k chain_matches" \
  "st:200:TOUED_LIB=${E}A2C_STAMPS_1.so python tools/a2c_stamps.py" \
  "gputest:900:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:500:python bench.py" \
  "trace:300:bash tools/trace_step.sh r04g" \
  "prof:900:bash tools/profile.sh r04g"
