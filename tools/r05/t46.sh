#!/bin/bash
# Round 5: the random sampler on a rank's agent slice against the full batch (both paths), then the full -m gpu suite
bash tools/gpu_steps.sh r05t46 \
  "par:300:python -u -m pytest tests/test_gpu_sampler.py -q -x --timeout 300 --timeout-method thread" \
  "gputest:900:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread"
