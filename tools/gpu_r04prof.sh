#!/bin/bash
# Round 4 (prof): kernel trace + stats of the headline and the C3/C4 workloads, FETCH/WRITE PMC passes and their
# calibration, of the final tree
bash tools/gpu_steps.sh r04prof "prof:1000:bash tools/profile.sh r04final"
