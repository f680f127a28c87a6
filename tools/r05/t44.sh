#!/bin/bash
# Round 5: k_embed_bwd3 with e2_w on the matrix cores too (EMBED_E2W_MFMA=1) against lane accumulators, and at 4 waves
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python tools/bench_embed.py --blocks 768,1024,1536"
bash tools/gpu_steps.sh r05t44 \
  "emb:300:TOUED_LIB=${E}EMBED_V_1.so $B --save gpurun_out/r05t44/g1.pt && $B --save gpurun_out/r05t44/g3.pt && TOUED_LIB=${E}EMBED_WPE_4.so $B && TOUED_LIB=${E}EMBED_E2W_MFMA_0.so $B && python -c \"import torch; a=torch.load('gpurun_out/r05t44/g1.pt'); b=torch.load('gpurun_out/r05t44/g3.pt'); print('v3 vs v1 rel', float((a-b).norm()/a.norm()), 'max', float((a-b).abs().max()))\"" \
  "par:400:python -u -m pytest tests/test_gpu_meta.py -q -x --timeout 300 --timeout-method thread -k 'meta_step_matches or one_launch or embed'"
