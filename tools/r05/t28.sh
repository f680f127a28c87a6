#!/bin/bash
# Round 5: localise the slab-h_in meta-gradient error
bash tools/gpu_steps.sh r05t28 \
  "wg:200:python -u -m pytest tests/test_gpu_wgrad.py -q --timeout 200 --timeout-method thread" \
  "meta:300:python -u -m pytest tests/test_gpu_meta.py -q --timeout 200 --timeout-method thread" \
  "full:300:python -u -m pytest tests/test_gpu_fullsize.py -q --timeout 200 --timeout-method thread"
