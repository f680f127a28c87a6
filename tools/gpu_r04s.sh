#!/bin/bash
# Round 4 (s): the A2C chain at a 168-VGPR budget (A2C_WAVES_PER_EU=3) so the side stream's draws kernels can be
# resident beside its two workgroups per CU: C3 bench and regret-round trace, A/B against the default build
E=to-ued_amd/exp/libtoued_
bash tools/gpu_steps.sh r04s \
  "c3_base:300:python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_w3:300:TOUED_LIB=${E}A2C_WAVES_PER_EU_3.so python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_base2:300:python bench.py --no_cpu_baseline --workloads c3 --steps 4" \
  "c3_w3b:300:TOUED_LIB=${E}A2C_WAVES_PER_EU_3.so python bench.py --no_cpu_baseline --workloads c3 --steps 4"
