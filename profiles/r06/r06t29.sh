#!/bin/bash
# Round 6, call 29: the round's profiles on the final tree -- kernel trace + stats of the headline bench and of the
# C3 / C4 workloads, FETCH_SIZE / WRITE_SIZE PMC passes with their calibration (tools/profile.sh)
bash tools/gpu_steps.sh r06t29 "prof:1100:bash tools/profile.sh r06f"
