#!/bin/bash
# Round 6, call 13: the round's profiles on the current tree -- kernel trace + stats of the headline bench and of the
# C3 / C4 workloads, FETCH_SIZE / WRITE_SIZE PMC passes with their calibration (tools/profile.sh), the SQ counter
# passes over the GRU, reduction and rollout micro-benchmarks (tools/pmc_kernels.sh)
bash tools/gpu_steps.sh r06t13 \
  "prof:1100:bash tools/profile.sh r06" \
  "sq:600:bash tools/pmc_kernels.sh r06"
