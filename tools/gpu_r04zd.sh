#!/bin/bash
# Round 4 (zd): the self-drawing A2C chain's draw waves at wave priority 0 (A2C_SELF_PRIO, default) against 3 (the
# env chain's): A2C tests, C3 A/B against the default chunked chain
E=to-ued_amd/exp/libtoued_
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_steps.sh r04zd \
  "plr:400:TOUED_A2C_SELF=1 $T tests/test_gpu_plr.py -k 'chain or regret'" \
  "c3_p0:300:TOUED_A2C_SELF=1 python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_old:300:python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_p3:300:TOUED_A2C_SELF=1 TOUED_LIB=${E}A2C_SELF_PRIO_3.so python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_p0b:300:TOUED_A2C_SELF=1 python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_oldb:300:python bench.py --no_cpu_baseline --workloads c3 --steps 4"
