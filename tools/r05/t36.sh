#!/bin/bash
# Round 5: k_embed_bwd3 (one lane per sample, e1_w / e1_b on the f32 MFMA) against k_embed_bwd: parity, timing, C2
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python tools/bench_embed.py --blocks 768,1024,1536,2048"
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t36 \
  "emb:300:TOUED_LIB=${E}EMBED_V_1.so $B --save gpurun_out/r05t36/g1.pt && $B --save gpurun_out/r05t36/g3.pt && TOUED_LIB=${E}EMBED_WPE_2.so $B && python -c \"import torch; a=torch.load('gpurun_out/r05t36/g1.pt'); b=torch.load('gpurun_out/r05t36/g3.pt'); print('v3 vs v1 rel', float((a-b).norm()/a.norm()), 'max', float((a-b).abs().max()))\"" \
  "par:400:python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_debug.py -q -x --timeout 200 --timeout-method thread" \
  "c2:400:TOUED_LIB=${E}EMBED_V_1.so $C && $C && TOUED_LIB=${E}EMBED_V_1.so $C && $C"
