#!/bin/bash
# Round 5: the one-launch reverse step with agents past their lifetime (HvpOp drops their samples): the bit-identity
# test (now with such agents) and the curve test that caught it, then the full -m gpu suite
bash tools/gpu_steps.sh r05t40 \
  "par:400:python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_curve.py -q -x --timeout 300 --timeout-method thread -k 'one_launch or certified'" \
  "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
