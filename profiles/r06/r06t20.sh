#!/bin/bash
# Round 6, call 20: the reverse step's fused kernel taking agents from a queue (agents of workgroups held off by the key
# chain's waves go to resident workgroups): bit identity against the previous commit, the fallback and bit-identity
# tests, block spans, and the C2 bench with and without the queue (the previous library runs with TOUED_ROWS_QUEUE=0:
# its toued_entropy_clip_hvp has no queue argument, and the stream argument is then NULL, the dump's stream)
H=$(pwd)/to-ued_amd/exp/libtoued_head.so
E=$(pwd)/to-ued_amd/exp/libtoued_
O=gpurun_out/r06t20
D="python tools/ab_dump.py"
C="python bench.py --workloads none --no_cpu_baseline --steps 10"
bash tools/gpu_steps.sh r06t20 \
  "dump:300:TOUED_ROWS_QUEUE=0 TOUED_LIB=$H $D dump $O/h.pt dense 64 5 && $D dump $O/n.pt dense 64 5 && TOUED_ROWS_QUEUE=0 TOUED_LIB=$H $D dump $O/hs.pt sparse 64 5 && $D dump $O/ns.pt sparse 64 5" \
  "cmp:120:$D compare $O/h.pt $O/n.pt; $D compare $O/hs.pt $O/ns.pt; rm -f $O/*.pt" \
  "tests:600:python -u -m pytest tests/test_gpu_fallbacks.py tests/test_gpu_meta.py -x -q --timeout 300 --timeout-method thread" \
  "rst:300:TOUED_LIB=${E}ROWS_STAMPS_1.so python tools/rows_stamps.py" \
  "c2:500:$C && TOUED_ROWS_QUEUE=0 $C && $C && TOUED_ROWS_QUEUE=0 $C"
