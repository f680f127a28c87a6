#!/bin/bash
# Round 5: bisect test_meta_return_curve_certified[0-7]'s step-1 meta-gradient error over the round's new paths
E=$(pwd)/to-ued_amd/exp/libtoued_
P="python -u -m pytest tests/test_gpu_curve.py -q -x --timeout 300 --timeout-method thread -k 'certified and 0-7'"
bash tools/gpu_steps.sh r05t39 \
  "ring0:300:TOUED_HIST_RING=0 $P" \
  "pack0:300:TOUED_PACK_SIDE=0 $P" \
  "pair0:300:TOUED_REVERSE_PAIR=0 $P" \
  "samp0:300:TOUED_SAMPLE_FUSED=0 $P" \
  "emb1:300:TOUED_LIB=${E}EMBED_V_1.so $P" \
  "ent0:300:TOUED_STEP_ENTROPY=0 $P"
