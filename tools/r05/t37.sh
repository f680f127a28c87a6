#!/bin/bash
# Round 5: the reverse pass's entropy-clip + HVP of step k in one launch (toued_entropy_clip_hvp) and the random
# sampler's key plumbing in one launch (toued_sample_random_keys): parity, C2 A/B
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
O="TOUED_REVERSE_PAIR=0 TOUED_SAMPLE_FUSED=0"
bash tools/gpu_steps.sh r05t37 \
  "par:400:python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_sampler.py -q -x --timeout 200 --timeout-method thread -k 'one_launch or fused_agent_step or meta_step_matches or backward or sample'" \
  "c2:500:$O $C && $C && $O $C && $C && $O $C && $C"
