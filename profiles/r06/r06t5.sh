#!/bin/bash
# Round 6, call 5: forward-save coverage on the unit-quad layout
bash tools/gpu_steps.sh r06t5 "fwd:200:python tools/det_fwd.py 4 2 && python tools/det_fwd.py 8 5"
